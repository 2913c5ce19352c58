"""Trained-weight files (``Weights/*.txt``, ``Results/*/*.txt``) and sharing expansion.

File format (writer ``Print_Functions.py:74-96``): line 1 ``"s0 s1 s2"`` (sharing of the CN,
UCN and VN weights), a blank line, then for every weight kind i with ``s_i > 0`` a block of
one tab-separated row per iteration followed by a blank line.  A row holds 1 value
(sharing 3), M or N values (sharing 2) or E values (sharing 1/4, edges in E(C) order).

Two readers are provided:

* ``read_weight_file``: format-aware, blocks are identified from the header line.
* ``load_weights_reference_order``: the reference's own row-counter reader semantics
  (``weight_init``, ``Main_Functions.py:387-439``), which reads rows according to the
  *current* sharing configuration and ``training_iter_start`` rather than the header.

``expand_weights`` turns per-kind rows into the per-iteration tables the decoder consumes:
``alpha[T, E]`` (CN weight per proto edge), ``alpha_ucn[T, E]`` (weight of edges whose check
was unsatisfied at the previous iteration) and ``beta[T, N]`` (VN weight on the channel LLR),
following the branches of ``Main_Functions.py:167-174`` and ``:266-304``.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

__all__ = ["WeightFile", "read_weight_file", "load_weights_reference_order",
           "expand_weights", "DecoderWeights", "flat_weights"]


@dataclass
class WeightFile:
    sharing: tuple
    blocks: Dict[int, np.ndarray]      # kind -> [rows, width] float64


def _parse_row(line: str) -> np.ndarray:
    return np.array([float(x) for x in line.replace("\t", " ").split()], dtype=np.float64)


def read_weight_file(path: str) -> WeightFile:
    with open(path) as f:
        lines = f.read().split("\n")
    sharing = tuple(int(x) for x in lines[0].split())
    if len(sharing) != 3:
        raise ValueError(f"{path}: bad sharing header {lines[0]!r}")
    blocks: Dict[int, np.ndarray] = {}
    pos = 1
    for kind, s in enumerate(sharing):
        if s <= 0:
            continue
        while pos < len(lines) and not lines[pos].strip():
            pos += 1
        rows = []
        while pos < len(lines) and lines[pos].strip():
            rows.append(_parse_row(lines[pos]))
            pos += 1
        if not rows:
            raise ValueError(f"{path}: missing block for weight kind {kind}")
        width = {len(r) for r in rows}
        if len(width) != 1:
            raise ValueError(f"{path}: ragged rows in block {kind}")
        blocks[kind] = np.stack(rows)
    return WeightFile(sharing, blocks)


def _kind_width(kind: int, share_type: int, M: int, N: int, E: int) -> int:
    if share_type in (1, 4):
        return E
    if share_type in (2, 5):
        return M if kind in (0, 1) else N
    if share_type == 3:
        return 1
    raise ValueError(f"unknown sharing type {share_type}")


def load_weights_reference_order(path: str, sharing, training_iter_start: int,
                                 training_iter_end: int, fixed_iter: int,
                                 M: int, N: int, E: int,
                                 init_weight: float = 1.0, init_vn_weight: float = 1.0):
    """Per-kind weight rows as ``weight_init`` builds them (``Main_Functions.py:387-439``).

    Rows for iterations ``t < training_iter_start`` come from the file, read by the same
    physical-line counter as the reference (``np.loadtxt(..., skiprows=1+row_idx)``);
    later iterations get the constant initial value (``init_weight`` / ``init_VN_weight``).
    Returns ``{kind: [n_iter, width] float32}``.
    """
    with open(path) as f:
        lines = f.read().split("\n")
    out = {}
    row_idx = 0
    for kind, s in enumerate(sharing):
        if s <= 0:
            continue
        width = _kind_width(kind, s, M, N, E)
        init = init_vn_weight if kind == 2 else init_weight
        n_iter = training_iter_end if s in (1, 2, 3) else fixed_iter + 1
        rows = []
        for t in range(n_iter):
            if t < training_iter_start:
                row_idx += 1
                # np.loadtxt(skiprows=1+row_idx, max_rows=1) skips physical lines, then
                # blank lines, and reads the next non-empty line.
                p = 1 + row_idx
                while p < len(lines) and not lines[p].strip():
                    p += 1
                if p >= len(lines):
                    raise ValueError(f"{path}: ran out of rows (kind {kind}, iteration {t})")
                vals = _parse_row(lines[p])
                if vals.size == 1:
                    vals = np.full(width, vals[0])
                if vals.size != width:
                    raise ValueError(f"{path}: row width {vals.size} != {width}")
                rows.append(vals.astype(np.float32))
            else:
                rows.append(np.full(width, init, np.float32))
        row_idx += 1
        out[kind] = np.stack(rows)
    return out


@dataclass
class DecoderWeights:
    """Per-iteration weight tables consumed by the decoder (all float32)."""
    alpha: np.ndarray                  # [T, E]   CN weight, E(C) edge order
    alpha_ucn: Optional[np.ndarray]    # [T, E]   weight on UCN edges, or None (UCN off)
    beta: np.ndarray                   # [T, N]   VN weight on the channel LLR

    @property
    def T(self) -> int:
        return int(self.alpha.shape[0])

    @property
    def ucn(self) -> bool:
        return self.alpha_ucn is not None


def _rows_from_file_block(block: np.ndarray, share_type: int, width: int, T: int,
                          fixed_iter: int) -> np.ndarray:
    block = np.asarray(block, np.float64).astype(np.float32)
    if block.shape[1] == 1 and width != 1:
        block = np.repeat(block, width, axis=1)
    if block.shape[1] != width:
        raise ValueError(f"weight row width {block.shape[1]} != expected {width}")
    out = np.empty((T, width), np.float32)
    for t in range(T):
        src = t if (share_type != 4 or t < fixed_iter) else fixed_iter
        if src >= block.shape[0]:
            raise ValueError(f"weight block has {block.shape[0]} rows, iteration {t} needs row {src}")
        out[t] = block[src]
    return out


def expand_weights(sharing, rows: Dict[int, np.ndarray], T: int, graph,
                   fixed_iter: int = 0) -> DecoderWeights:
    """Expand per-kind rows (``{kind: [rows, width]}``) to per-iteration tables.

    CN branch (``Main_Functions.py:266-304``): type 0 -> |o| unweighted (alpha = 1, which is
    bit-identical since |o|*1.0f == |o|); 1 -> per edge; 2 -> per check row i (``var @
    W_skipconn2odd``); 3 -> scalar; 4 -> per edge, iterations >= fixed_iter reuse row
    ``fixed_iter``.  Type 5 has no CN branch in the reference (it raises), so it is rejected.
    UCN weights are used only for the pairs (1,1), (2,2), (3,3).
    VN branch (``Main_Functions.py:167-174``): 2 -> per column j; 3 -> scalar; 4 -> like CN
    type 4; any other type leaves the channel unweighted.
    """
    s0, s1, s2 = (int(x) for x in sharing)
    E, M, N = graph.E, graph.M, graph.N
    pe_row = graph.pe_row

    def cn_table(kind, s):
        if s == 0:
            return np.ones((T, E), np.float32)
        if s == 5:
            raise ValueError("CN sharing type 5 is not implemented by the reference decoder")
        width = _kind_width(kind, s, M, N, E)
        r = _rows_from_file_block(rows[kind], s, width, T, fixed_iter)
        if s == 2:
            return np.ascontiguousarray(r[:, pe_row])
        if s == 3:
            return np.repeat(r[:, :1], E, axis=1)
        return r

    alpha = cn_table(0, s0)
    alpha_ucn = None
    if s1 > 0 and s0 == s1 and s0 in (1, 2, 3):
        alpha_ucn = cn_table(1, s1)
    if s2 in (2, 3, 4):
        width = _kind_width(2, s2, M, N, E)
        b = _rows_from_file_block(rows[2], s2, width, T, fixed_iter)
        beta = b if s2 != 3 else np.repeat(b[:, :1], N, axis=1)
        if beta.shape[1] != N:
            raise ValueError("VN weight width mismatch")
    else:
        beta = np.ones((T, N), np.float32)
    return DecoderWeights(np.ascontiguousarray(alpha, np.float32),
                          None if alpha_ucn is None else np.ascontiguousarray(alpha_ucn, np.float32),
                          np.ascontiguousarray(beta, np.float32))


def flat_weights(graph, T: int, alpha: float = 1.0, beta: float = 1.0,
                 alpha_ucn: Optional[float] = None) -> DecoderWeights:
    """Constant weights (e.g. the flat [3,0,3] alpha=0.75, beta=1 configuration)."""
    a = np.full((T, graph.E), alpha, np.float32)
    u = None if alpha_ucn is None else np.full((T, graph.E), alpha_ucn, np.float32)
    b = np.full((T, graph.N), beta, np.float32)
    return DecoderWeights(a, u, b)
