"""Quasi-cyclic base graphs, code parameters and the lifted Tanner graph.

Replaces the reference's host-side graph construction:

* ``load_base_graph``  <- ``np.loadtxt("./BaseGraph/{name}.txt", int, delimiter='\\t')``
  (``main_Base.py:67``).
* ``CodeParams``        <- ``init_parameter`` (``Main_Functions.py:8-38``), including the
  rate quirk of ``Main_Functions.py:24-29``: ``punct_num = pe - ps + 1`` and
  ``short_num = se - ss + 1`` are subtracted even when the ranges are ``0..0``.
* ``TannerGraph``       <- ``init_connecting_matrix`` (``Main_Functions.py:46-150``).  The
  reference encodes the lifted graph as dense 0/1 matrices (two (E*z)^2 cyclic-shift
  permutations plus E x E / N x E gathers).  Here the same graph is a sorted edge list:
  lifted edge (e, h) of proto edge e = (i, j) joins check ``i*z + h`` to variable
  ``j*z + ((h + P[i,j] mod z) mod z)`` (``Main_Functions.py:64-66,72-74``); proto edges are
  numbered in the row-major order E(C) that the reference uses for per-edge weights and
  for ``LLRa`` (``Main_Functions.py:69-71``).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

__all__ = ["load_base_graph", "CodeParams", "TannerGraph", "snr_to_sigma", "code_rate"]


def load_base_graph(path: str) -> np.ndarray:
    """Read a ``BaseGraph/*.txt`` proto matrix: tab-separated ints, -1 = no edge."""
    proto = np.loadtxt(path, dtype=np.int64, delimiter="\t", ndmin=2)
    if proto.ndim != 2 or proto.size == 0:
        raise ValueError(f"{path}: not a 2-D proto matrix")
    return proto


def code_rate(proto: np.ndarray, z: int, punct_start: int = 0, punct_end: int = 0,
              short_start: int = 0, short_end: int = 0) -> float:
    """Rate exactly as ``Main_Functions.py:24-29`` computes it (quirk included)."""
    M, N = proto.shape
    punct_num = punct_end - punct_start + 1
    short_num = short_end - short_start + 1
    n = N * z - punct_num - short_num
    k = (N - M) * z - short_num
    return 1.0 * k / n


def snr_to_sigma(snr_db, rate: float) -> np.ndarray:
    """sigma = sqrt(1 / (2 * 10^(EbN0/10) * rate))  (``Main_Functions.py:35-36``), float64."""
    snr = np.asarray(snr_db, dtype=np.float64)
    lin = 10.0 ** (snr / 10.0)
    return np.sqrt(1.0 / (2.0 * lin * rate))


@dataclass
class CodeParams:
    """Scalars of ``init_parameter`` (``Main_Functions.py:8-38``)."""
    proto: np.ndarray
    z: int
    punct_start: int = 0
    punct_end: int = 0
    short_start: int = 0
    short_end: int = 0

    def __post_init__(self):
        self.proto = np.asarray(self.proto, dtype=np.int64)
        base = (self.proto != -1).astype(np.int64)
        self.M, self.N = self.proto.shape
        self.base = base
        self.cn_deg = base.sum(axis=1)
        self.vn_deg = base.sum(axis=0)
        self.E = int(self.vn_deg.sum())
        self.rate = code_rate(self.proto, self.z, self.punct_start, self.punct_end,
                              self.short_start, self.short_end)

    def sigma(self, snr_db) -> np.ndarray:
        return snr_to_sigma(snr_db, self.rate)


@dataclass
class TannerGraph:
    """Lifted Tanner graph of a QC proto matrix as sorted edge lists.

    Lifted edges are stored check-major: the edges of check ``c = i*z + h`` occupy rows
    ``z*row_off[i] + h*deg[i] + k`` for k = 0..deg[i]-1, k following ascending column j
    (this is the order the HIP kernels use for message rows).
    """
    proto: np.ndarray
    z: int
    M: int = field(init=False)
    N: int = field(init=False)
    E: int = field(init=False)

    def __post_init__(self):
        P = np.asarray(self.proto, dtype=np.int64)
        self.proto = P
        self.M, self.N = P.shape
        z = self.z
        rows, cols = np.nonzero(P != -1)            # row-major == E(C) order
        self.pe_row = rows.astype(np.int64)
        self.pe_col = cols.astype(np.int64)
        self.pe_shift = (P[rows, cols] % z).astype(np.int64)
        self.E = int(rows.size)
        self.cn_deg = np.bincount(rows, minlength=self.M).astype(np.int64)
        self.vn_deg = np.bincount(cols, minlength=self.N).astype(np.int64)
        self.row_ptr = np.concatenate([[0], np.cumsum(self.cn_deg)]).astype(np.int64)
        # position of each proto edge inside its row
        self.pe_k = np.arange(self.E) - self.row_ptr[rows]
        # E(V) order (column-major, Main_Functions.py:61-63) -> E(C) index
        order_v = np.lexsort((rows, cols))
        self.ev_to_ec = order_v.astype(np.int64)
        self.n_checks = self.M * z
        self.n_vars = self.N * z
        self.n_edges = self.E * z
        self._build_lifted()

    def _build_lifted(self):
        z = self.z
        n_edges = self.n_edges
        edge_check = np.empty(n_edges, np.int64)
        edge_var = np.empty(n_edges, np.int64)
        edge_pe = np.empty(n_edges, np.int64)
        for i in range(self.M):
            d = int(self.cn_deg[i])
            base = z * int(self.row_ptr[i])
            pes = np.arange(self.row_ptr[i], self.row_ptr[i + 1])
            for h in range(z):
                r0 = base + h * d
                edge_check[r0:r0 + d] = i * z + h
                edge_var[r0:r0 + d] = self.pe_col[pes] * z + (h + self.pe_shift[pes]) % z
                edge_pe[r0:r0 + d] = pes
        self.edge_check = edge_check
        self.edge_var = edge_var
        self.edge_pe = edge_pe
        self.check_ptr = np.empty(self.n_checks + 1, np.int64)
        self.check_ptr[:-1] = np.searchsorted(edge_check, np.arange(self.n_checks))
        self.check_ptr[-1] = n_edges
        self.max_check_deg = int(self.cn_deg.max()) if self.M else 0
        self.max_var_deg = int(self.vn_deg.max()) if self.N else 0
        # variable-side adjacency: edges of variable v, sorted by check
        order = np.lexsort((edge_check, edge_var))
        self.var_edges = order
        self.var_ptr = np.concatenate([[0], np.cumsum(np.bincount(edge_var, minlength=self.n_vars))])

    # ---- dense helpers (tests / fixtures only; small graphs) ------------------------
    def parity_check_matrix(self) -> np.ndarray:
        """Dense lifted H [M*z, N*z] as uint8 (for tests on small codes)."""
        H = np.zeros((self.n_checks, self.n_vars), np.uint8)
        H[self.edge_check, self.edge_var] = 1
        return H

    def padded_check_edges(self):
        """[n_checks, max_check_deg] edge rows, -1 padded."""
        out = -np.ones((self.n_checks, self.max_check_deg), np.int64)
        deg = np.diff(self.check_ptr)
        for d in np.unique(deg):
            cs = np.nonzero(deg == d)[0]
            out[cs, :d] = self.check_ptr[cs][:, None] + np.arange(d)[None, :]
        return out

    def padded_var_edges(self):
        """[n_vars, max_var_deg] edge rows (sorted by check), -1 padded."""
        out = -np.ones((self.n_vars, self.max_var_deg), np.int64)
        deg = np.diff(self.var_ptr)
        for v in range(self.n_vars):
            d = deg[v]
            out[v, :d] = self.var_edges[self.var_ptr[v]:self.var_ptr[v] + d]
        return out


def default_graph_dir() -> str:
    """Directory holding BaseGraph/*.txt files (``LDPC_DATA_DIR`` overrides)."""
    here = os.path.dirname(os.path.abspath(__file__))
    return os.environ.get("LDPC_DATA_DIR", os.path.join(here, "data"))
