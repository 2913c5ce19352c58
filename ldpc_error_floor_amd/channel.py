"""Host-side AWGN channel and uncorrected-word file I/O (the parity-mode input source).

* ``quantize_host``       <- ``Cal_MSA_Q``      (``Print_Functions.py:12-25``), float64 numpy.
* ``create_mix_epoch``    <- same name          (``Print_Functions.py:29-72``).  The
  reference loops per codeword with ``np.vstack`` (O(B^2) copying); this version draws the
  identical random streams vectorized: for every codeword the word RNG is advanced by
  ``randint(0, 2, N*z)`` (its value is discarded for the all-zero word) and the noise RNG
  supplies ``normal(0, 1, N*z)``; the two RandomStates are independent so drawing them
  as [B, N*z] blocks consumes them identically.
* ``read_uncor_llr`` / ``write_uncor_file`` <- same names (``Print_Functions.py:6-10``,
  ``:120-126``); ``load_uncor_inputs`` <- ``process_data`` (``Main_Functions.py:526-576``).
"""
from __future__ import annotations

import os

import numpy as np

__all__ = ["quantize_host", "create_mix_epoch", "read_uncor_llr", "write_uncor_file",
           "append_uncor_rows", "load_uncor_inputs"]


def quantize_host(x, q_bit: int):
    """q-bit QMS quantizer on the host (round half to even, then clip)."""
    x = np.asarray(x)
    if q_bit == 6:
        return np.clip(np.round(x), -15.5, 15.5)
    if q_bit == 5:
        return np.clip(np.round(x * 2) / 2, -7.5, 7.5)
    if q_bit == -5:
        return np.clip(np.round(x), -15, 15)
    if q_bit == 4:
        return np.clip(np.round(x), -7, 7)
    if q_bit == 3:
        return np.clip(np.round(x / 2) * 2, -6, 6)
    raise ValueError(f"unsupported q_bit {q_bit}")


def create_mix_epoch(scaling_factor, wordRandom, noiseRandom, batch_size, code_n, code_k, Z,
                     code_GM, is_zeros_word, decoding_type, punct_start, punct_end,
                     short_start, short_end, q_bit, clip_LLR):
    """AWGN LLR batch with the reference's exact RNG consumption (log p1/p0 convention).

    Returns ``X`` float64 [B, code_n, Z] and ``Y`` int64 [B, code_n*Z] like the reference.
    Codeword b uses ``scaling_factor[b % len(scaling_factor)]`` (the reference cycles the
    SNR list per codeword).
    """
    if not is_zeros_word:
        raise NotImplementedError("only the all-zero codeword is supported "
                                  "(the reference passes code_GM=[] and trains on zeros)")
    sf = np.atleast_1d(np.asarray(scaling_factor, dtype=np.float64))
    n = code_n * Z
    B = int(batch_size)
    wordRandom.randint(0, 2, size=(B, n))                       # advanced, value unused
    noise = noiseRandom.normal(0.0, 1.0, (B, n))
    sig = sf[np.arange(B) % sf.size][:, None]
    X_p = noise * sig + (-1.0)                                   # Y = 0 -> BPSK -1
    llr = 2 * X_p / (sig ** 2)
    if decoding_type == 2:
        llr = quantize_host(llr, q_bit)
    if punct_start > 0:
        llr[:, punct_start - 1:punct_end] = 0.001 if decoding_type == 0 else 0
    if short_start > 0:
        llr[:, short_start - 1:short_end] = -clip_LLR
    X = llr.reshape(B, code_n, Z)
    Y = np.zeros((B, n), dtype=np.int64)
    return X, Y


def read_uncor_llr(input_llr, input_codeword, batch_idx, batch_size, code_n, Z):
    X = -np.reshape(input_llr[batch_idx * batch_size:(batch_idx + 1) * batch_size, ...],
                    [batch_size, code_n, Z])
    Y = input_codeword[batch_idx * batch_size:(batch_idx + 1) * batch_size, :]
    return X, Y


def write_uncor_file(uncor_flag, training_received_data, code_length, path="Uncor.txt"):
    """Append frames with ``uncor_flag == 1`` as 3 zero columns + negated LLRs (``%.1f``)."""
    sel = np.asarray(uncor_flag) == 1
    num = int(np.sum(sel))
    append_uncor_rows(np.reshape(np.asarray(training_received_data)[sel, :, :], [num, code_length]),
                      path)


def append_uncor_rows(llr_rows, path="Uncor.txt", formatter=None):
    """The row format of ``write_uncor_file`` (``Print_Functions.py:120-126``) for LLR rows
    [n, N*z] already selected (e.g. collected on the GPU by ``NMSDecoder.collect_uncorrected``).
    ``formatter``: a callable rows -> the same text as bytes (the native
    ``NMSDecoder.format_uncor_rows``, ~10x np.savetxt's rate); None = np.savetxt."""
    if formatter is not None:
        data = formatter(np.ascontiguousarray(llr_rows, np.float32))
        with open(path, "ab") as f:
            f.write(data)
        return
    rows = np.asarray(llr_rows, np.float64)
    num = rows.shape[0]
    with open(path, "a") as f:
        np.savetxt(f, np.concatenate((np.zeros((num, 3)), -rows), axis=1), fmt="%.1f",
                   delimiter="\t")


def load_uncor_inputs(filename, training_num, valid_flag, valid_num, test_flag, test_num,
                      inputs_dir="./Inputs"):
    """``process_data`` for ``sampling_type == 1`` (raises instead of ``sys.exit``)."""
    def load(suffix, num):
        path = os.path.join(inputs_dir, f"[Uncor]_{filename}{suffix}.txt")
        arr = np.loadtxt(path, dtype=np.float32, delimiter="\t")
        if arr.ndim > 1:
            arr = np.delete(arr, [0, 1, 2], 1)
        if arr.shape[0] < num:
            raise ValueError(f"Wrong input: {path} has {arr.shape[0]} rows < {num}")
        arr = arr[:num]
        return arr, np.zeros(arr.shape, dtype=np.int64)

    tr, trc = load("", training_num)
    va, vac = load("_Valid", valid_num) if valid_flag == 1 else ([], [])
    te, tec = load("_Test", test_num) if test_flag == 1 else ([], [])
    return tr, trc, va, vac, te, tec
