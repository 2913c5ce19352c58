"""ORACLE — test infrastructure only.  CPU restatement of the on-GPU AWGN channel.

Only ``tests/`` may import this module, as the checker of ``ldpc_channel_awgn`` /
``ldpc_decode_awgn`` (``ldpc_error_floor_amd/csrc/ldpc_awgn.h``).  The product path never
calls it.

What it restates.  The GPU channel is the build's throughput-mode replacement of the
reference's host channel ``create_mix_epoch`` (``/root/reference/Print_Functions.py:29-72``):
the same channel model for the all-zero codeword (BPSK 0 -> -1, y = sigma n - 1,
LLR = 2 y / sigma^2 in the log p1/p0 convention of ``:45-46``, ``Cal_MSA_Q`` quantization of
``:12-25`` in QMS mode, punctured bits -> 0 (0.001 for sum-product) and shortened bits ->
-clip_LLR after quantization, ``:52-66``), with the numpy ``RandomState`` normal stream
replaced by a counter-based one:

  * Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as 1, 2, 3",
    SC'11; the Random123 library's ``philox4x32_R(10, ...)``), key = the 64-bit seed
    (low word, high word), counter = (pair index pr, global codeword index low / high word,
    tag 0x4C445043).  ``philox4x32_10`` is pinned by the published Random123 known-answer
    vectors (``tests/test_philox_oracle.py``).
  * float modes (sum-product, MS): Box-Muller per pair of bits (2 pr, 2 pr + 1) of a
    codeword: u1 from 53 bits ((c0 << 21) ^ (c1 >> 11)), u1 = (fp32(m53) + 0.5) 2^-53 in
    (0, 1]; u2 = (fp32(c2) + 0.5) 2^-32; r = sqrt(-2 log u1); n = (r cos 2 pi u2,
    r sin 2 pi u2); then the fp32 channel steps (no fused multiply-add: the library is built
    with -ffp-contract=off).
  * QMS (every q_bit): the quantized LLR is sampled as its level directly.  ``qms_levels``
    restates the host's ``awgn_qms_levels`` (``csrc/ldpc_host.cpp``): Cal_MSA_Q's levels, the
    LLR rounding boundaries x_j between them, n_j = (x_j sigma^2 / 2 + 1) / sigma and the
    64-bit thresholds T_j = floor(2^64 Phi(n_j)) (from the upper tail, 2^64 - floor(2^64 (1 -
    Phi(n_j))), when n_j >= 0), Phi from ``math.erfc`` (the same libm erfc the library calls).
    Element (codeword at global index gb, variable v): U = hi << 32 | lo with hi = word gb mod 4
    of Philox(v, gb div 4, 'LDQ4') and lo = the same word of Philox(v, gb div 4, 'LDQR'); its
    level = #{j : U >= T_j}.  (The device draws lo only when hi equals some T_j's high word;
    the comparison is the same.)

Precision contract.  Philox and the two uniforms are integer / exactly-rounded and match the
GPU bit for bit.  QMS LLRs are integer comparisons against thresholds both sides compute with
the same double operations and libm erfc, so they agree bit for bit.  Float-mode ``logf`` and
``sincospif`` are the device math library's (within a couple of ulps of the correctly rounded
value computed here), so float LLRs agree to a few ulps.
"""
from __future__ import annotations

import numpy as np

__all__ = ["philox4x32_10", "awgn_normals", "awgn_llr", "quantize_f32", "near_boundary",
           "qms_levels", "awgn_qms_levels", "awgn_qms_llr", "awgn_q8"]

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = 0x9E3779B9
W1 = 0xBB67AE85
TAG = 0x4C445043
TAG_Q = 0x4C445134          # 'LDQ4': high words of the QMS uniforms
TAG_R = 0x4C445152          # 'LDQR': their low words
QUANT = {6: (1.0, 15.5), 5: (0.5, 7.5), -5: (1.0, 15.0), 4: (1.0, 7.0), 3: (2.0, 6.0)}
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """Philox4x32 with 10 rounds.  ctr: uint32 array [..., 4]; key: (k0, k1) ints or uint32
    arrays broadcastable to ctr[..., 0].  Returns uint32 [..., 4]."""
    c = [np.asarray(ctr[..., i], dtype=np.uint64) for i in range(4)]
    k0 = np.asarray(key[0], dtype=np.uint64) & MASK32
    k1 = np.asarray(key[1], dtype=np.uint64) & MASK32
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c = [hi1 ^ c[1] ^ k0, lo1, hi0 ^ c[3] ^ k1, lo0]
        k0 = (k0 + np.uint64(W0)) & MASK32
        k1 = (k1 + np.uint64(W1)) & MASK32
    return np.stack([x.astype(np.uint32) for x in c], axis=-1)


def _f32_of_uint(x):
    """fp32(x) for a uint64 below 2^53, round to nearest even (exact via float64)."""
    return np.asarray(x, np.uint64).astype(np.float64).astype(np.float32)


def awgn_normals(B, n_vars, seed, offset=0):
    """Standard normals [B, n_vars] float32 of codewords offset .. offset+B-1 (global index)."""
    npairs = (n_vars + 1) // 2
    gcw = (np.uint64(offset) + np.arange(B, dtype=np.uint64))[:, None]
    pr = np.arange(npairs, dtype=np.uint64)[None, :]
    ctr = np.empty((B, npairs, 4), np.uint32)
    ctr[..., 0] = pr
    ctr[..., 1] = (gcw & MASK32).astype(np.uint32)
    ctr[..., 2] = (gcw >> np.uint64(32)).astype(np.uint32)
    ctr[..., 3] = TAG
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c = philox4x32_10(ctr, (seed & 0xFFFFFFFF, seed >> 32)).astype(np.uint64)
    m53 = ((c[..., 0] << np.uint64(21)) ^ (c[..., 1] >> np.uint64(11))) & np.uint64((1 << 53) - 1)
    u1 = (_f32_of_uint(m53) + np.float32(0.5)) * np.float32(2.0 ** -53)
    u2 = (_f32_of_uint(c[..., 2]) + np.float32(0.5)) * np.float32(2.0 ** -32)
    # correctly rounded fp32 logf / sqrtf / sincospif (the device's are within ulps of these)
    lg = np.log(u1.astype(np.float64)).astype(np.float32)
    r = np.sqrt(np.float32(-2.0) * lg)
    ang = np.float32(2.0) * u2                   # exact (power-of-two scaling)
    cs = np.cos(np.pi * ang.astype(np.float64)).astype(np.float32)
    sn = np.sin(np.pi * ang.astype(np.float64)).astype(np.float32)
    nz = np.stack([r * cs, r * sn], axis=-1).reshape(B, 2 * npairs)
    return nz[:, :n_vars]


def quantize_f32(x, q_bit):
    """awgn_quant in fp32 (Cal_MSA_Q, Print_Functions.py:12-25)."""
    x = np.asarray(x, np.float32)
    if q_bit == 6:
        return np.clip(np.rint(x), -15.5, 15.5).astype(np.float32)
    if q_bit == 5:
        return np.clip(np.rint(x * np.float32(2)) * np.float32(0.5), -7.5, 7.5).astype(np.float32)
    if q_bit == -5:
        return np.clip(np.rint(x), -15, 15).astype(np.float32)
    if q_bit == 4:
        return np.clip(np.rint(x), -7, 7).astype(np.float32)
    return np.clip(np.rint(x * np.float32(0.5)) * np.float32(2), -6, 6).astype(np.float32)


def qms_levels(sigma, q_bit):
    """(T uint64 [nb] ascending, level values float32 [nb + 1], kmin) of ``awgn_qms_levels``
    (csrc/ldpc_host.cpp): Cal_MSA_Q's levels (Print_Functions.py:12-25) and the 64-bit CDF
    thresholds of their rounding boundaries for LLR = 2 (sigma n - 1) / sigma^2 (:29-72)."""
    import math
    u, cmax = QUANT[q_bit]
    K = int(math.ceil(cmax / u)) + 1
    Q = lambda k: min(max(k * u, -cmax), cmax)           # noqa: E731
    vals, thr = [Q(-K)], []
    s2 = float(sigma) * float(sigma)
    for k in range(-K + 1, K + 1):
        if Q(k) == Q(k - 1):
            continue
        x = (k - 0.5) * u
        nz = (x * s2 * 0.5 + 1.0) / float(sigma)
        if nz < 0.0:
            T = int(math.ldexp(0.5 * math.erfc(-nz * 0.7071067811865476), 64))
        else:
            tail = int(math.ldexp(0.5 * math.erfc(nz * 0.7071067811865476), 64))
            T = (1 << 64) - 1 if tail == 0 else (1 << 64) - tail
        thr.append(T)
        vals.append(Q(k))
    kmin = 0 if q_bit == 6 else int(round(-cmax / u))
    return np.array(thr, np.uint64), np.array(vals, np.float32), kmin


def _qms_uniforms(B, n_vars, seed, offset):
    """64-bit uniforms [B, n_vars] of codewords offset .. offset + B - 1 (global index)."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    key = (seed & 0xFFFFFFFF, seed >> 32)
    gb = np.uint64(offset) + np.arange(B, dtype=np.uint64)
    gq = (gb >> np.uint64(2))[:, None]
    j = (gb & np.uint64(3)).astype(np.int64)
    v = np.arange(n_vars, dtype=np.uint64)[None, :]
    ctr = np.empty((B, n_vars, 4), np.uint32)
    ctr[..., 0] = v
    ctr[..., 1] = (gq & MASK32).astype(np.uint32)
    ctr[..., 2] = (gq >> np.uint64(32)).astype(np.uint32)
    ctr[..., 3] = TAG_Q
    hi = np.take_along_axis(philox4x32_10(ctr, key), j[:, None, None].repeat(n_vars, 1), 2)[..., 0]
    ctr[..., 3] = TAG_R
    lo = np.take_along_axis(philox4x32_10(ctr, key), j[:, None, None].repeat(n_vars, 1), 2)[..., 0]
    return (hi.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)


def awgn_qms_levels(B, n_vars, sigma, seed, offset=0, q_bit=5):
    """Level indices int [B, n_vars] (0 .. nb) of the QMS sampler, before puncture / shorten."""
    T, _, _ = qms_levels(sigma, q_bit)
    U = _qms_uniforms(B, n_vars, seed, offset)
    return np.searchsorted(T, U, side="right")


def _fixed(n_vars, punct, short):
    bit = np.arange(1, n_vars + 1)
    pm = (bit >= punct[0]) & (bit <= punct[1]) if punct[0] > 0 else np.zeros(n_vars, bool)
    sm = (bit >= short[0]) & (bit <= short[1]) if short[0] > 0 else np.zeros(n_vars, bool)
    return pm, sm


def awgn_qms_llr(B, n_vars, sigma, seed, offset=0, q_bit=5, punct=(0, 0), short=(0, 0), clip=20.0):
    """QMS LLRs float32 [B, n_vars] as ldpc_channel_awgn (decoding_type 2)."""
    _, vals, _ = qms_levels(sigma, q_bit)
    llr = vals[awgn_qms_levels(B, n_vars, sigma, seed, offset, q_bit)]
    pm, sm = _fixed(n_vars, punct, short)
    llr[:, pm] = np.float32(0.0)
    llr[:, sm] = -np.float32(clip)
    return llr


def awgn_q8(B, n_vars, sigma, seed, offset=0, q_bit=5, punct=(0, 0), short=(0, 0)):
    """ldpc_decode_awgn's byte channel (the bytes the bit-sliced kernels' prologue generates,
    gen_bytes in ldpc_bs_kernel.h) uint8 [ceil(B/32)][n_vars][32]: byte r of
    (pack, v) = grid value + 16 of codeword 32 pack + r (rows past B generated too), 16 on a
    punctured bit, 48 - qmax on a shortened one (the bit-sliced kernels' marker)."""
    npk = (B + 31) // 32
    _, _, kmin = qms_levels(sigma, q_bit)
    lv = awgn_qms_levels(npk * 32, n_vars, sigma, seed, offset, q_bit)
    byte = (lv + 16 + kmin).astype(np.uint8)
    pm, sm = _fixed(n_vars, punct, short)
    byte[:, pm] = 16
    byte[:, sm] = 48 + kmin            # kmin = -qmax
    return np.ascontiguousarray(byte.reshape(npk, 32, n_vars).transpose(0, 2, 1))


def awgn_llr(B, n_vars, sigma, seed, offset=0, decoding_type=2, q_bit=5, punct=(0, 0),
             short=(0, 0), clip=20.0):
    """(LLR float32 [B, n_vars], unquantized LLR float32 [B, n_vars] or None for QMS) as
    ldpc_channel_awgn."""
    if decoding_type == 2:
        return awgn_qms_llr(B, n_vars, sigma, seed, offset, q_bit, punct, short, clip), None
    sig = np.float32(sigma)
    inv = np.float32(2.0 / (float(sigma) * float(sigma)))
    nz = awgn_normals(B, n_vars, seed, offset)
    raw = ((nz * sig) - np.float32(1.0)) * inv
    llr = raw.copy()
    pm, sm = _fixed(n_vars, punct, short)
    llr[:, pm] = np.float32(0.001 if decoding_type == 0 else 0.0)
    llr[:, sm] = -np.float32(clip)
    return llr, raw


def near_boundary(raw, q_bit, rel=1e-5):
    """Elements whose unquantized value lies within ``rel`` (relative, plus the same absolute)
    of a rounding boundary of the q-bit grid: there an ulp-level difference in logf /
    sincospif can move the quantized value by one step."""
    raw = np.asarray(raw, np.float64)
    unit = {6: 1.0, 5: 0.5, -5: 1.0, 4: 1.0, 3: 2.0}[q_bit]
    g = raw / unit
    frac = np.abs(g - np.floor(g) - 0.5)
    return frac * unit <= rel * (1.0 + np.abs(raw))
