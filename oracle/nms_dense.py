"""ORACLE / CPU BASELINE — test & bench infrastructure only (see oracle/nms_oracle.py header).

Dense "TF-graph-equivalent" numpy restatement of the reference decoder, used as the CPU
baseline in bench.py (``cpu_baseline.kind = "port"``).  TensorFlow is not installable here,
so this reproduces the reference graph's *cost structure* op for op on numpy/BLAS: per
iteration the same dense (E*z)^2 cyclic-shift permutation matmuls (Main_Functions.py:192,
203, 219, 261), the same [B, z, E, E] tiled min / product reductions (:231-254) and the same
proto-level gather matmuls (:213-214, :317).  Numerically it is the same algorithm as
nms_oracle.decode (QMS results are bit-identical; tests check that).
"""
from __future__ import annotations

import numpy as np

from .nms_oracle import quantize

F32 = np.float32


class DenseGraph:
    """Dense matrices of the reference formulation, built from the proto matrix."""

    def __init__(self, proto, z):
        P = np.asarray(proto, np.int64)
        self.M, self.N = P.shape
        self.z = z
        r_c, c_c = np.nonzero(P != -1)                       # E(C): row-major
        ev = np.lexsort((r_c, c_c))                          # E(V) order -> E(C) index
        E = r_c.size
        self.E = E
        s_c = P[r_c, c_c] % z
        ec_of_ev = ev
        ev_of_ec = np.empty(E, np.int64)
        ev_of_ec[ec_of_ev] = np.arange(E)
        Ez = E * z
        h = np.arange(z)
        L1 = np.zeros((Ez, Ez), F32)                         # blocks in E(V) order
        L2 = np.zeros((Ez, Ez), F32)                         # blocks in E(C) order
        for k in range(E):
            s_v = s_c[ec_of_ev[k]]
            L1[k * z + h, k * z + (h + s_v) % z] = 1
            L2[k * z + h, k * z + (h + s_c[k]) % z] = 1
        self.L1T = np.ascontiguousarray(L1.T)
        self.L2 = L2
        same_col = c_c[:, None] == c_c[None, :]
        same_row = r_c[:, None] == r_c[None, :]
        eye = np.eye(E, dtype=bool)
        # VN extrinsic [E(C), E(V)]: sum of the other edges of the column
        self.W_v = ((same_col & ~eye)[:, ec_of_ev]).astype(F32)
        # channel -> edges [N, E(V)]
        self.W_ch = (np.arange(self.N)[:, None] == c_c[ec_of_ev][None, :]).astype(F32)
        # CN extrinsic mask, flattened like the tiled graph: [E(C) out, E(V) in]
        self.mask_cn = ((same_row & ~eye)[:, ec_of_ev]).astype(F32).reshape(-1)
        self.mask_cn_self = ((same_row)[:, ec_of_ev]).astype(F32).reshape(-1)
        # edges -> VN sum [E(C), N]
        self.W_out = (c_c[:, None] == np.arange(self.N)[None, :]).astype(F32)
        self.W_row = (np.arange(self.M)[:, None] == r_c[None, :]).astype(F32)   # [M, E(C)]


def _lift(x, L, B, E, z):
    """[B, z, E] -> E-major flatten -> @ L -> [B, z, E]."""
    y = np.transpose(x, (0, 2, 1)).reshape(B, E * z) @ L
    return np.transpose(y.reshape(B, E, z), (0, 2, 1))


def decode(llr, proto, z, alpha, alpha_ucn, beta, T=None, decoding_type=2, q_bit=5, clip=20.0,
           graph=None):
    """Same signature / outputs (``app`` only) as nms_oracle.decode, dense formulation."""
    g = graph if graph is not None else DenseGraph(proto, z)
    E, N, M = g.E, g.N, g.M
    T = alpha.shape[0] if T is None else T
    ch = np.asarray(llr, F32).reshape(-1, N, z)
    B = ch.shape[0]
    qms = decoding_type == 2
    clipf = F32(clip)
    xa_t = np.transpose(ch, (0, 2, 1))                                   # [B, z, N]
    c2v = np.zeros((B, z, E), F32)                                       # E(C)
    apps = np.empty((T, B, N * z), F32)
    app_prev = None
    for t in range(T):
        lw = xa_t * beta[t].astype(F32)
        if qms:
            lw = quantize(lw, q_bit)
        ucn = None
        if alpha_ucn is not None:
            src = lw if t == 0 else np.transpose(app_prev.reshape(B, N, z), (0, 2, 1))
            sgn = np.where(-src > 0, F32(1), F32(-1))
            e_sgn = _lift(sgn @ g.W_ch, g.L1T, B, E, z)
            tile = np.tile(e_sgn, (1, 1, E)) * g.mask_cn_self
            tile = tile + (1 - (np.abs(tile) > 0))
            prod = tile.reshape(B, z, E, E).prod(axis=3)
            ucn = (prod < 0).astype(F32)
            ucn = _lift(ucn, g.L2, B, E, z)
        x2 = lw @ g.W_ch + c2v @ g.W_v
        x2 = _lift(x2, g.L1T, B, E, z)
        x2 = quantize(x2, q_bit) if qms else np.clip(x2, -clipf, clipf)
        if decoding_type in (1, 2):
            x2 = x2 + F32(1e-4) * (1 - (np.abs(x2) > 0))
        x21 = (np.tile(x2, (1, 1, E)) * g.mask_cn).reshape(B, z, E, E)
        mag = np.abs(x21) + F32(10000) * (1 - (np.abs(x21) > 0))
        x3 = mag.min(axis=3)
        x3 = x3 + F32(-1e-4) * (1 - (np.abs(x3) > F32(1e-4)))
        x4 = 1 - 2 * (-x21 < 0)
        o = x3 * np.sign(-np.prod(x4, axis=3)).astype(F32)
        o = _lift(o.astype(F32), g.L2, B, E, z)
        w = (alpha[t].astype(F32))[None, None, :]
        x = np.abs(o) * w
        if ucn is not None:
            xu = np.abs(o) * alpha_ucn[t].astype(F32)[None, None, :]
            x = x * (1 - ucn) + xu * ucn
        x = x * (x > 0)
        x = quantize(x, q_bit) if qms else np.clip(x, -clipf, clipf)
        c2v = (x * np.sign(o)).astype(F32)
        S = np.transpose(c2v @ g.W_out, (0, 2, 1))                       # [B, N, z]
        chq = quantize(ch, q_bit) if qms else ch
        app = np.clip(chq + S, -clipf, clipf).reshape(B, N * z)
        apps[t] = app
        app_prev = app
    return dict(app=apps)
