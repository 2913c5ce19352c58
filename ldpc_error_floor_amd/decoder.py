"""``NMSDecoder``: the HIP decoder over torch device tensors.

This is the build's replacement for the T-iteration graph that ``build_neural_network``
unrolls (``Main_Functions.py:157-385``) and ``compute_results`` runs through ``sess.run``
(``Print_Functions.py:147-151``).  Inputs are LLRs ``[B, N*z]`` (or ``[B, N, z]``, the
``xa`` placeholder shape) in the reference's log(p1/p0) convention; outputs are
``ya_output_all`` (``[T*B, Nt*z]`` float32), per-iteration hard bits / syndromes, and
on-device FER/BER counters.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _native
from .code import TannerGraph
from .config import DECODING_MS, DECODING_MS_NONUDGE, DECODING_QMS, DECODING_SP, VALID_Q_BITS
from .weights import DecoderWeights

__all__ = ["NMSDecoder", "Decoder", "DecodeResult", "KERNELS"]

KERNELS = {"auto": 0, "flood": 1, "fused": 2}


@dataclass
class DecodeResult:
    app: Optional["object"] = None          # torch f32 [T, B, Nt*z]
    hard: Optional["object"] = None         # torch int32 [T, B, ceil(N*z/32)] (bit words)
    synd: Optional["object"] = None         # torch int32 [T, B, ceil(M*z/32)]
    counters: Optional["object"] = None     # torch int64 [4]
    flags: Optional["object"] = None        # torch uint8 [B]
    iter_wrong: Optional["object"] = None   # torch int32 [T, ceil(B/32)]: bit b%32 of word
                                            # (t, b//32) = frame b wrong at iteration t

    def frame_errors(self, B: int) -> np.ndarray:
        """``iter_wrong`` unpacked on the host: bool [T, B] (calc_ber_fer's per-iteration frame
        error, ``Print_Functions.py:100-118``)."""
        return unpack_bits(self.iter_wrong.cpu().numpy(), B).astype(bool)

    def ya_output_all(self):
        """``ya_output_all`` layout: iterations stacked on axis 0 -> [T*B, Nt*z]."""
        T, B, n = self.app.shape
        return self.app.reshape(T * B, n)


def unpack_bits(words, n_bits: int) -> np.ndarray:
    """[..., W] uint32 words (bit k of word w = bit 32w+k) -> [..., n_bits] uint8."""
    w = np.ascontiguousarray(np.asarray(words).astype(np.uint32))
    b = np.unpackbits(w.view(np.uint8).reshape(w.shape + (4,)), axis=-1, bitorder="little")
    return b.reshape(w.shape[:-1] + (w.shape[-1] * 32,))[..., :n_bits]


class NMSDecoder:
    def __init__(self, proto, z: int, weights: DecoderWeights, decoding_type: int = DECODING_QMS,
                 q_bit: int = 5, target_node: int = 0, clip_LLR: float = 20.0, device=None,
                 kernel: str = "auto", B_max: int = 0):
        import torch
        self._torch = torch
        if decoding_type not in (DECODING_SP, DECODING_MS, DECODING_QMS, DECODING_MS_NONUDGE):
            raise ValueError(f"decoding_type {decoding_type} not supported")
        if decoding_type == DECODING_QMS and q_bit not in VALID_Q_BITS:
            raise ValueError(f"q_bit {q_bit} not in {VALID_Q_BITS}")
        if kernel not in KERNELS:
            raise ValueError(f"kernel must be one of {list(KERNELS)}")
        self.graph = TannerGraph(np.asarray(proto), int(z))
        self.z = int(z)
        self.N, self.M = self.graph.N, self.graph.M
        self.n_vars = self.N * self.z
        self.n_checks = self.M * self.z
        self.target_node = int(target_node) if target_node and target_node > 0 else self.N
        self.target_bits = self.target_node * self.z
        self.decoding_type = int(decoding_type)
        self.q_bit = int(q_bit)
        self.clip = float(clip_LLR)
        self.kernel = kernel
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("NMSDecoder runs on a ROCm GPU device only (no CPU fallback)")
        self._ext = _native.load()
        self._g = self._ext.Graph(self.graph.proto.astype(np.int32), self.z,
                                  self.device.index or 0)
        self.set_weights(weights)
        self._ctx = None
        self._ctx_B = 0
        self._ctx_T = 0
        if B_max:
            self._ensure_ctx(B_max, self.T)

    # ------------------------------------------------------------------------------
    def set_weights(self, weights: DecoderWeights):
        W = weights
        if W.alpha.shape[1] != self.graph.E or W.beta.shape[1] != self.N:
            raise ValueError("weight tables do not match the graph")
        self.weights = W
        self.T = W.T
        self._g.set_weights(np.ascontiguousarray(W.alpha, np.float32),
                            None if W.alpha_ucn is None else np.ascontiguousarray(W.alpha_ucn, np.float32),
                            np.ascontiguousarray(W.beta, np.float32))

    def _ensure_ctx(self, B: int, T: int):
        if self._ctx is None or B > self._ctx_B or T > self._ctx_T:
            Bm = max(B, self._ctx_B)
            Tm = max(T, self._ctx_T, self.T)
            self._ctx = None
            self._ctx = self._ext.Ctx(self._g, int(Bm), int(Tm))
            self._ctx_B, self._ctx_T = Bm, Tm
        return self._ctx

    def kernel_info(self, T=None, kernel=None):
        T = self.T if T is None else T
        ctx = self._ensure_ctx(1, T)
        return self._ext.kernel_info(ctx, T, self.decoding_type, self.q_bit, self.target_bits,
                                     KERNELS[kernel or self.kernel], self.clip)

    def supports(self, kernel: str, T=None) -> bool:
        try:
            self.kernel_info(T, kernel)
            return True
        except RuntimeError:
            return False

    def _as_llr(self, llr):
        torch = self._torch
        if not isinstance(llr, torch.Tensor):
            llr = torch.from_numpy(np.ascontiguousarray(np.asarray(llr, np.float32)))
        llr = llr.to(device=self.device, dtype=torch.float32)
        B = llr.shape[0]
        if B == 0:
            return llr.reshape(0, self.n_vars)
        llr = llr.reshape(B, -1).contiguous()
        if llr.shape[1] != self.n_vars:
            raise ValueError(f"llr has {llr.shape[1]} bits per codeword, graph has {self.n_vars}")
        return llr

    def decode(self, llr, T: Optional[int] = None, app: bool = True, hard: bool = False,
               synd: bool = False, counters=None, flags: bool = False, kernel: Optional[str] = None,
               stream=None, target_bits: Optional[int] = None, iter_wrong: bool = False) -> DecodeResult:
        """Decode a batch.  ``counters`` may be a caller-owned int64[4] device tensor that is
        accumulated into (``+=``); pass ``True`` to get a fresh one.  ``target_bits``
        overrides the output / FER bit range (default Nt*z).  ``iter_wrong``: the per-iteration
        frame-error words (every kernel, the counters-only ones included)."""
        torch = self._torch
        T = self.T if T is None else int(T)
        nt = self.target_bits if target_bits is None else int(target_bits)
        if T > self.T:
            raise ValueError(f"T={T} exceeds the {self.T} iterations the weights cover")
        llr = self._as_llr(llr)
        B = int(llr.shape[0])
        if B == 0:
            return self._empty_result(T, nt, hard, synd, counters, flags, app, iter_wrong)
        ctx = self._ensure_ctx(B, T)
        res = DecodeResult()
        dev = self.device
        if app:
            res.app = torch.empty((T, B, nt), dtype=torch.float32, device=dev)
        if hard:
            res.hard = torch.empty((T, B, (self.n_vars + 31) // 32), dtype=torch.int32, device=dev)
        if synd:
            res.synd = torch.empty((T, B, (self.n_checks + 31) // 32), dtype=torch.int32, device=dev)
        if counters is True:
            counters = torch.zeros(4, dtype=torch.int64, device=dev)
        if counters is not None:
            if counters.dtype != torch.int64 or counters.numel() < 4 or counters.device != dev:
                raise ValueError("counters must be an int64[4] tensor on the decoder's device")
            res.counters = counters
        if isinstance(flags, torch.Tensor):                 # caller-owned uint8 [>= B]
            if flags.dtype != torch.uint8 or flags.device != dev or flags.numel() < B:
                raise ValueError("flags tensor must be uint8 on the decoder's device, >= B long")
            res.flags = flags
        elif flags:
            res.flags = torch.empty(B, dtype=torch.uint8, device=dev)
        if iter_wrong:
            res.iter_wrong = torch.empty((T, (B + 31) // 32), dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
        self._ext.decode(ctx, llr.data_ptr(), B, T, self.decoding_type, self.q_bit,
                         nt, self.clip, KERNELS[kernel or self.kernel],
                         ptr(res.app), ptr(res.hard), ptr(res.synd), ptr(res.counters),
                         ptr(res.flags), stream.cuda_stream, ptr(res.iter_wrong))
        return res

    def generates_channel_in_kernel(self, T=None, kernel=None, app: bool = False) -> bool:
        """Whether a counters-only ``decode_awgn`` (``app``: one with an APP export) generates
        the LLRs inside the decoding kernel (the prologue of the fused v5 kernel, and of the
        bit-sliced kernels for QMS counters-only decodes); otherwise ``ldpc_decode_awgn`` runs
        the channel kernel into HBM and then the decoder (flood, ffl).  The C ABI's own decision
        (``ldpc_awgn_in_kernel``), with this decoder's shortened range."""
        T = self.T if T is None else T
        ctx = self._ensure_ctx(1, T)
        short = getattr(self, "short", (0, 0)) or (0, 0)
        return bool(self._ext.awgn_in_kernel(ctx, T, self.decoding_type, self.q_bit, self.target_bits,
                                             KERNELS[kernel or self.kernel], self.clip,
                                             has_short=short[0] > 0, app=app))

    def last_kernel(self) -> str:
        """The kernel that served this decoder's last decode (``ldpc_ctx_last_kernel``)."""
        return "" if self._ctx is None else self._ext.last_kernel(self._ctx)

    def _empty_result(self, T, nt, hard, synd, counters, flags, app, iter_wrong=False):
        """An empty batch decodes to empty outputs; a caller's counters are left unchanged."""
        torch = self._torch
        dev = self.device
        res = DecodeResult()
        if app:
            res.app = torch.empty((T, 0, nt), dtype=torch.float32, device=dev)
        if hard:
            res.hard = torch.empty((T, 0, (self.n_vars + 31) // 32), dtype=torch.int32, device=dev)
        if synd:
            res.synd = torch.empty((T, 0, (self.n_checks + 31) // 32), dtype=torch.int32, device=dev)
        if counters is True:
            counters = torch.zeros(4, dtype=torch.int64, device=dev)
        res.counters = counters if counters is not None else None
        if isinstance(flags, torch.Tensor):
            res.flags = flags[:0]
        elif flags:
            res.flags = torch.empty(0, dtype=torch.uint8, device=dev)
        if iter_wrong:
            res.iter_wrong = torch.empty((T, 0), dtype=torch.int32, device=dev)
        return res

    def decode_awgn(self, B: int, sigma: float, seed: int, offset: int = 0, punct=None, short=None,
                    T: Optional[int] = None, app: bool = False, counters=None, flags=None,
                    kernel: Optional[str] = None, stream=None, iter_wrong: bool = False) -> DecodeResult:
        """Decode B codewords whose LLRs come from the on-GPU AWGN channel, generated inside
        the decoder (``ldpc_decode_awgn``): identical to ``decode(awgn(...))`` without the
        LLRs ever being written to HBM.  ``counters`` / ``flags`` as in ``decode``."""
        torch = self._torch
        T = self.T if T is None else int(T)
        punct = getattr(self, "punct", (0, 0)) if punct is None else punct
        short = getattr(self, "short", (0, 0)) if short is None else short
        if int(B) == 0:
            return self._empty_result(T, self.target_bits, False, False, counters, flags, app, iter_wrong)
        ctx = self._ensure_ctx(int(B), T)
        dev = self.device
        res = DecodeResult()
        if app:
            res.app = torch.empty((T, B, self.target_bits), dtype=torch.float32, device=dev)
        if counters is True:
            counters = torch.zeros(4, dtype=torch.int64, device=dev)
        if counters is not None:
            if counters.dtype != torch.int64 or counters.numel() < 4 or counters.device != dev:
                raise ValueError("counters must be an int64[4] tensor on the decoder's device")
            res.counters = counters
        if isinstance(flags, torch.Tensor):
            if flags.dtype != torch.uint8 or flags.device != dev or flags.numel() < B:
                raise ValueError("flags tensor must be uint8 on the decoder's device, >= B long")
            res.flags = flags
        elif flags:
            res.flags = torch.empty(B, dtype=torch.uint8, device=dev)
        if iter_wrong:
            res.iter_wrong = torch.empty((T, (int(B) + 31) // 32), dtype=torch.int32, device=dev)
        if stream is None:
            stream = torch.cuda.current_stream(dev)
        ptr = lambda t: 0 if t is None else t.data_ptr()   # noqa: E731
        self._ext.decode_awgn(ctx, int(B), T, self.decoding_type, self.q_bit, self.target_bits,
                              self.clip, KERNELS[kernel or self.kernel], float(sigma), int(seed),
                              int(offset), int(punct[0]), int(punct[1]), int(short[0]),
                              int(short[1]), ptr(res.app), ptr(res.counters), ptr(res.flags),
                              stream.cuda_stream, ptr(res.iter_wrong))
        return res

    def _uncorrected_index(self, flags, stream):
        """Batch indices (sorted, on the device) of the frames wrong at every iteration."""
        torch = self._torch
        B = int(flags.shape[0])
        idx = torch.empty(max(B, 1), dtype=torch.int64, device=self.device)
        cnt = torch.empty(1, dtype=torch.int64, device=self.device)
        self._ext.collect_frames(flags.data_ptr(), B, 1, 1, idx.data_ptr(), B, cnt.data_ptr(),
                                 stream.cuda_stream)
        stream.synchronize()
        n = int(cnt.item())
        return torch.sort(idx[:n]).values.contiguous()     # batch order, as the reference writes

    def collect_uncorrected(self, flags, llr, stream=None):
        """LLR rows (host float32 [n, N*z], batch order) of the frames wrong at every iteration
        (``frame_flags`` bit 0 = the reference's ``uncor_flag``), compacted on the GPU by
        ``ldpc_collect_frames`` + ``ldpc_gather_rows``; only the n rows cross PCIe."""
        torch = self._torch
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        sel = self._uncorrected_index(flags, stream)
        n = int(sel.numel())
        if n == 0:
            return np.zeros((0, self.n_vars), np.float32)
        llr = llr.reshape(llr.shape[0], -1)
        rows = torch.empty((n, self.n_vars), dtype=torch.float32, device=self.device)
        for s0 in range(0, n, 65535):
            s1 = min(n, s0 + 65535)
            self._ext.gather_rows(llr.data_ptr(), self.n_vars, sel[s0:].data_ptr(), s1 - s0,
                                  rows[s0:].data_ptr(), stream.cuda_stream)
        return rows.cpu().numpy()

    def collect_uncorrected_awgn(self, flags, sigma: float, seed: int, offset: int = 0,
                                 punct=None, short=None, stream=None):
        """``collect_uncorrected`` after ``decode_awgn``: the failing frames' LLR rows
        regenerated from the channel (``ldpc_channel_awgn_rows``, the same values ``awgn`` would
        have written), so the sweep keeps the in-kernel channel while collecting."""
        torch = self._torch
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        punct = getattr(self, "punct", (0, 0)) if punct is None else punct
        short = getattr(self, "short", (0, 0)) if short is None else short
        with torch.cuda.stream(stream):          # (allocations and the copy on `stream`)
            sel = self._uncorrected_index(flags, stream)
            n = int(sel.numel())
            if n == 0:
                return np.zeros((0, self.n_vars), np.float32)
            rows = torch.empty((n, self.n_vars), dtype=torch.float32, device=self.device)
            self._ext.channel_awgn_rows(rows.data_ptr(), sel.data_ptr(), n, self.n_vars, float(sigma),
                                        int(seed), int(offset), self.decoding_type, self.q_bit,
                                        int(punct[0]), int(punct[1]), int(short[0]), int(short[1]),
                                        self.clip, stream.cuda_stream)
            return rows.cpu().numpy()

    def format_uncor_rows(self, rows):
        """``write_uncor_file``'s text for float32 LLR rows [n, N*z] as bytes, formatted by the
        native ``ldpc_format_uncor_rows`` (byte-identical to np.savetxt with "%.1f")."""
        return self._ext.format_uncor_rows(rows)

    def awgn(self, B: int, sigma: float, seed: int, offset: int = 0, punct=None, short=None,
             out=None, stream=None):
        """On-GPU AWGN LLRs [B, N*z] for the all-zero word (Philox, see ldpc_channel.hip).
        ``punct`` / ``short`` default to the ranges the decoder was built with (``Decoder``)."""
        torch = self._torch
        punct = getattr(self, "punct", (0, 0)) if punct is None else punct
        short = getattr(self, "short", (0, 0)) if short is None else short
        if out is None:
            out = torch.empty((B, self.n_vars), dtype=torch.float32, device=self.device)
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        self._ext.channel_awgn(out.data_ptr(), int(B), self.n_vars, float(sigma), int(seed),
                               int(offset), self.decoding_type, self.q_bit, int(punct[0]),
                               int(punct[1]), int(short[0]), int(short[1]), self.clip,
                               stream.cuda_stream)
        return out


def Decoder(graph_txt: str, z: int, punct=(0, 0), short=(0, 0), sharing=(3, 0, 3),
            decoding_type: int = DECODING_QMS, q_bit: int = 5, weights_txt: Optional[str] = None,
            T: Optional[int] = None, target_node: int = 0, fixed_iter: int = 0,
            clip_LLR: float = 20.0, device=None, kernel: str = "auto", B_max: int = 0) -> NMSDecoder:
    """File-level constructor (SURVEY §8 b): a base-graph text file (``BaseGraph/*.txt``, read
    like ``init_parameter``, ``Main_Functions.py:8-38``) and a weights file
    (``Weights/*.txt``, ``Main_Functions.py:387-439``) -> an ``NMSDecoder``.

    ``punct`` / ``short`` are the 1-based inclusive ranges of ``create_mix_epoch``
    (``Print_Functions.py:29-72``); they belong to the channel, so they only become the
    defaults of ``awgn``.  ``T`` defaults to the number of iterations the weight file holds;
    without a weight file the decoder uses flat weights (alpha 1, beta 1) for ``T`` iterations.
    """
    from .code import load_base_graph
    from .weights import expand_weights, read_weight_file, flat_weights
    proto = load_base_graph(graph_txt)
    g = TannerGraph(proto, int(z))
    if weights_txt is not None:
        wf = read_weight_file(weights_txt)
        if T is None:
            T = max(int(b.shape[0]) for b in wf.blocks.values()) if wf.blocks else 1
        W = expand_weights(tuple(sharing), wf.blocks, int(T), g, fixed_iter)
    else:
        if T is None:
            raise ValueError("T is required without a weights file")
        W = flat_weights(g, int(T))
    dec = NMSDecoder(proto, z, W, decoding_type, q_bit, target_node, clip_LLR, device=device,
                     kernel=kernel, B_max=B_max)
    dec.punct = (int(punct[0]), int(punct[1]))
    dec.short = (int(short[0]), int(short[1]))
    return dec
