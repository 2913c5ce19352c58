"""C-ABI library: loads, exports every symbol include/*.h declares (the decoder ABI
ldpc_nms.h and the test hooks of ldpc_nms_debug.h), and validates arguments before touching
the GPU (CPU only — no compute calls)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ldpc_nms.h")
HEADERS = sorted(os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include"))
                 if f.endswith(".h"))
LIB = os.path.join(ROOT, "ldpc_error_floor_amd", "libldpc_nms.so")


def declared_functions(headers=(HEADER,)):
    out = set()
    for hdr in headers:
        src = open(hdr).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        out |= set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(ldpc_\w+)\s*\(", src, flags=re.M))
    return sorted(out)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built: run python -m ldpc_error_floor_amd.build")
    return ctypes.CDLL(LIB)


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("ldpc_graph_create", "ldpc_graph_destroy", "ldpc_weights_set", "ldpc_ctx_create",
              "ldpc_ctx_destroy", "ldpc_decode", "ldpc_channel_awgn", "ldpc_kernel_info"):
        assert f in fns


def test_every_declared_symbol_is_exported(lib):
    fns = declared_functions(HEADERS)
    assert "ldpc_debug_bs_bounds" in fns and "ldpc_decode" in fns
    missing = [f for f in fns if not hasattr(lib, f)]
    assert not missing, missing


def test_version_and_status_strings(lib):
    assert lib.ldpc_abi_version() == 3
    lib.ldpc_status_string.restype = ctypes.c_char_p
    assert lib.ldpc_status_string(0) == b"ok"
    assert b"argument" in lib.ldpc_status_string(-1)
    assert lib.ldpc_status_string(-99) == b"unknown status"


def test_argument_validation_without_gpu(lib):
    out = ctypes.c_void_p()
    proto = (ctypes.c_int32 * 4)(0, -1, 1, 0)
    assert lib.ldpc_graph_create(None, 2, 2, 4, 0, ctypes.byref(out)) == -1
    assert lib.ldpc_graph_create(proto, 0, 2, 4, 0, ctypes.byref(out)) == -1
    assert lib.ldpc_graph_create(proto, 2, 2, 4, 0, None) == -1
    bad = (ctypes.c_int32 * 4)(-3, -1, 1, 0)
    assert lib.ldpc_graph_create(bad, 2, 2, 4, 0, ctypes.byref(out)) == -1
    assert lib.ldpc_graph_destroy(None) == -1
    assert lib.ldpc_ctx_destroy(None) == -1
    assert lib.ldpc_decode(None, None, 1, None, None, None) == -1
    assert lib.ldpc_ctx_create(None, 10, 10, ctypes.byref(out)) == -1
    buf = ctypes.create_string_buffer(16)
    assert lib.ldpc_ctx_last_kernel(None, buf, 16) == -1
    lib.ldpc_channel_awgn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                                      ctypes.c_double, ctypes.c_uint64, ctypes.c_int64] + \
        [ctypes.c_int32] * 6 + [ctypes.c_float, ctypes.c_void_p]
    assert lib.ldpc_channel_awgn(None, 4, 10, 0.5, 1, 0, 2, 5, 0, 0, 0, 0, 20.0, None) == -1


def test_row_writer_and_row_channel_validation_without_gpu(lib):
    """ldpc_format_uncor_rows checks its capacity and arguments; ldpc_channel_awgn_rows rejects
    bad arguments before any launch (and n = 0 is a no-op)."""
    import numpy as np
    f = lib.ldpc_format_uncor_rows
    f.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                  ctypes.POINTER(ctypes.c_int64)]
    rows = np.zeros((2, 3), np.float32)
    ln = ctypes.c_int64(-5)
    small = ctypes.create_string_buffer(10)
    assert f(rows.ctypes.data, 2, 3, small, 10, ctypes.byref(ln)) == -1 and ln.value == 0
    assert f(rows.ctypes.data, 2, 0, small, 10, ctypes.byref(ln)) == -1
    assert f(rows.ctypes.data, 2, 3, small, 10, None) == -1
    cap = 2 * (13 + 48 * 3)
    buf = ctypes.create_string_buffer(cap)
    assert f(rows.ctypes.data, 2, 3, buf, cap, ctypes.byref(ln)) == 0
    assert buf.raw[:ln.value] == b"0.0\t0.0\t0.0\t-0.0\t-0.0\t-0.0\n" * 2
    g = lib.ldpc_channel_awgn_rows
    g.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_double,
                  ctypes.c_uint64, ctypes.c_int64] + [ctypes.c_int32] * 6 + [ctypes.c_float, ctypes.c_void_p]
    assert g(None, None, 4, 10, 0.5, 1, 0, 2, 5, 0, 0, 0, 0, 20.0, None) == -1   # no buffers
    assert g(None, None, -1, 10, 0.5, 1, 0, 2, 5, 0, 0, 0, 0, 20.0, None) == -1  # n < 0
    assert g(None, None, 0, 10, -0.5, 1, 0, 2, 5, 0, 0, 0, 0, 20.0, None) == -1  # sigma <= 0
    assert g(None, None, 0, 10, 0.5, 1, 0, 2, 5, 0, 0, 0, 0, 20.0, None) == 0    # nothing to do
