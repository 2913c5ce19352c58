"""Test-only helpers: host counters from APP, and an oracle-backed stand-in decoder used to
exercise the host logic (Session, FER loops, sharding) on CPU.  Never used by the product."""
import ctypes
import os
from types import SimpleNamespace

import numpy as np

from oracle import nms_oracle


_LIB = None


def native_format_uncor_rows(rows):
    """``ldpc_format_uncor_rows`` of the C-ABI library (host code, no GPU) through ctypes."""
    global _LIB
    if _LIB is None:
        _LIB = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                        "ldpc_error_floor_amd", "libldpc_nms.so"))
        _LIB.ldpc_format_uncor_rows.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                                ctypes.c_void_p, ctypes.c_int64,
                                                ctypes.POINTER(ctypes.c_int64)]
    rows = np.ascontiguousarray(rows, np.float32)
    n, nc = rows.shape
    cap = n * (13 + 48 * nc)
    buf = ctypes.create_string_buffer(max(cap, 1))
    ln = ctypes.c_int64()
    st = _LIB.ldpc_format_uncor_rows(rows.ctypes.data, n, nc, buf, cap, ctypes.byref(ln))
    if st != 0:
        raise RuntimeError(f"ldpc_format_uncor_rows: {st}")
    return buf.raw[:ln.value]


def counters_from_app(app):
    """[T, B, Nt] APP -> int64[4] {bit errors @T-1, frames wrong @T-1, frames wrong at every t,
    2*loss} for the all-zero codeword (calc_ber_fer + loss_type 2 semantics)."""
    app = np.asarray(app)
    hd = app >= 0
    wrong = hd.any(axis=2)                      # [T, B]
    last = app[-1]
    pos = (last > 0).any(axis=1)
    return np.array([hd[-1].sum(), wrong[-1].sum(), wrong.all(axis=0).sum(),
                     2 * pos.sum() + (wrong[-1] & ~pos).sum()], np.int64)


def flags_from_app(app):
    hd = np.asarray(app) >= 0
    wrong = hd.any(axis=2)
    return (wrong.all(axis=0).astype(np.uint8) | (wrong[-1].astype(np.uint8) << 1))


class OracleDecoder:
    """Duck-types the parts of NMSDecoder that Session / fer_sweep use, on CPU."""

    def __init__(self, proto, z, W, decoding_type=2, q_bit=5, target_node=0):
        import torch
        self.torch = torch
        self.proto, self.z, self.W = np.asarray(proto), z, W
        self.M, self.N = self.proto.shape
        self.n_vars = self.N * z
        self.target_bits = (target_node or self.N) * z
        self.T = W.T
        self.dt, self.q = decoding_type, q_bit
        self.device = torch.device("cpu")
        self.g = nms_oracle.lifted_edges(self.proto, z)

    def decode(self, llr, T=None, app=True, counters=None, target_bits=None, kernel=None,
               flags=None, **kw):
        T = T or self.T
        x = np.asarray(llr.cpu().numpy() if hasattr(llr, "cpu") else llr, np.float32)
        out = nms_oracle.decode(x.reshape(x.shape[0], -1), self.proto, self.z, self.W.alpha,
                                self.W.alpha_ucn, self.W.beta, T, self.dt, self.q, graph=self.g)
        nt = target_bits or self.target_bits
        a = out["app"][:, :, :nt]
        if counters is not None:
            counters += self.torch.from_numpy(counters_from_app(a))
        if flags is not None and not isinstance(flags, bool):
            flags.copy_(self.torch.from_numpy(flags_from_app(a)))
        return SimpleNamespace(app=self.torch.from_numpy(np.ascontiguousarray(a)) if app else None)

    def collect_uncorrected(self, flags, llr):
        sel = (flags.cpu().numpy() & 1) == 1
        return np.asarray(llr.cpu().numpy(), np.float32).reshape(llr.shape[0], -1)[sel]

    def format_uncor_rows(self, rows):
        return native_format_uncor_rows(rows)

    def awgn(self, B, sigma, seed, offset=0, punct=(0, 0), short=(0, 0), out=None, **kw):
        # deterministic per global codeword index (like the GPU Philox stream)
        rows = []
        for b in range(B):
            rs = np.random.RandomState((seed * 1000003 + offset + b) % (2 ** 31))
            y = rs.normal(0, 1, self.n_vars) * sigma - 1.0
            rows.append(np.clip(np.round(2 * y / sigma ** 2 * 2) / 2, -7.5, 7.5))
        arr = self.torch.from_numpy(np.array(rows, np.float32))
        if out is not None:
            out.copy_(arr)
            return out
        return arr
