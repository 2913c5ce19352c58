"""ldpc_format_uncor_rows (the native writer of write_uncor_file's rows,
Print_Functions.py:120-126) is byte-identical to np.savetxt(fmt="%.1f", delimiter="\\t") of
3 zero columns + the negated float32 LLRs -- on random LLRs, exact half-tenth ties, signed
zeros, values that round to -0.0, subnormals, values past the 1e15 fast-path limit, inf and nan."""
import io
import os

import numpy as np
import pytest

from _helpers import native_format_uncor_rows
from ldpc_error_floor_amd.channel import append_uncor_rows


def _savetxt(rows):
    rows = np.asarray(rows, np.float64)
    f = io.BytesIO()
    np.savetxt(f, np.concatenate((np.zeros((rows.shape[0], 3)), -rows), axis=1), fmt="%.1f",
               delimiter="\t")
    return f.getvalue()


def _edge_values():
    k = np.arange(-400, 401)
    ties = k / 20.0                                  # x*10 exactly half-integer for odd k
    quarters = k / 4.0
    special = [0.0, -0.0, 0.04, -0.04, 0.05, -0.05, 0.0499999, -0.0500001, 0.25, -0.25, 0.75,
               1e-45, -1e-45, 1.17549435e-38, 999999999999999.9, 1e15, -1e15, 1.5e15, 3.4e38,
               -3.4e38, np.inf, -np.inf, np.nan, -np.nan, 7.5, -7.5, 20.0, -20.0, 123456.75]
    return np.concatenate([ties, quarters, special]).astype(np.float32)


@pytest.mark.parametrize("n_cols", [1, 7, 576])
def test_native_rows_match_savetxt(n_cols):
    rng = np.random.default_rng(n_cols)
    vals = np.concatenate([_edge_values(), (rng.normal(0, 8, 6000)).astype(np.float32),
                           (rng.normal(0, 1, 3000) * 10.0 ** rng.integers(-6, 12, 3000)).astype(np.float32),
                           rng.integers(-40, 41, 2000).astype(np.float32) / 2])
    n = len(vals) // n_cols
    rows = vals[:n * n_cols].reshape(n, n_cols)
    assert native_format_uncor_rows(rows) == _savetxt(rows)


def test_empty_and_append(tmp_path):
    assert native_format_uncor_rows(np.zeros((0, 5), np.float32)) == b""
    rows = np.random.default_rng(1).normal(0, 4, (33, 24)).astype(np.float32)
    a, b = tmp_path / "a.txt", tmp_path / "b.txt"
    for p, fmt in ((a, None), (b, native_format_uncor_rows)):
        append_uncor_rows(rows[:10], str(p), formatter=fmt)
        append_uncor_rows(rows[10:], str(p), formatter=fmt)
    assert a.read_bytes() == b.read_bytes() and os.path.getsize(a) > 0
