"""Host-side bounds check of the bit-sliced kernel's reads (CPU, no GPU): for every kBsInst
instance and UCN setting whose plan serves a graph (C2-C4 and every fixture graph of the
reference's BaseGraph/), the launch's own planning code builds its tables and every index the
kernel reads is checked against the allocation the context makes (ldpc_debug_bs_bounds,
csrc/ldpc_bs.hip bs_bounds_check).  The class it guards is the round-4 fault
(profiles/r4/README.md, r4c: one-chunk UCN instances read the check-lane hard-decision table for
the waves past cn_lanes, off the end of its allocation; the guard is ldpc_bs_kernel.h's
`ql < a.cn_lanes`): with the guard dropped (LDPC_BOUNDS_PRE_GUARD) the check must report it."""
import ctypes
import os

import numpy as np
import pytest

from conftest import ROOT
from ldpc_error_floor_amd.code import load_base_graph

LIB = os.path.join(ROOT, "ldpc_error_floor_amd", "libldpc_nms.so")
BG = os.path.join(ROOT, "ldpc_error_floor_amd", "data", "BaseGraph")
MODE = {5: 1, -5: 2, 4: 3, 3: 4}
PRE_GUARD = 1

# (graph file, z): the SURVEY 8 d workloads and the fixture graphs
GRAPHS = [("wman_N0576_R34_z24", 24), ("802_11n_N648_R56_z27", 27),
          ("5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640", 64),
          ("5G_LDPC_R0.73_n_dec2304_n2112_k1536_z72_s1537_1584", 72),
          ("5G_LDPC_R0.33_n_dec896_n768_k256_z32_s257_320", 32),
          ("5G_LDPC_R0.50_n_dec640_n512_k256_z32_s257_320", 32),
          ("5G_LDPC_R0.73_n_dec480_n352_k256_z32_s257_320", 32),
          ("MACKAY_N96_K48", 1), ("BCH_63_51", 1)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built: run python -m ldpc_error_floor_amd.build")
    L = ctypes.CDLL(LIB)
    L.ldpc_debug_bs_bounds.argtypes = [ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                       ctypes.c_int32, ctypes.c_float, ctypes.c_int32,
                                       ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_int32]
    return L


def bounds(lib, name, z, T, q=5, au=1, bu=1, flags=0, clip=20.0):
    P = np.ascontiguousarray(load_base_graph(os.path.join(BG, name + ".txt")), np.int32)
    v = ctypes.c_int32(-1)
    msg = ctypes.create_string_buffer(256)
    n = lib.ldpc_debug_bs_bounds(P.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), P.shape[0], P.shape[1],
                                 z, T, MODE[q], au, bu, clip, flags, ctypes.byref(v), msg, 256)
    return n, v.value, msg.value.decode()


@pytest.mark.parametrize("name,z", GRAPHS)
@pytest.mark.parametrize("au,bu", [(1, 1), (0, 0), (1, 0)])
@pytest.mark.parametrize("T", [20, 50])
def test_every_read_inside_its_allocation(lib, name, z, au, bu, T):
    n, v, msg = bounds(lib, name, z, T, au=au, bu=bu)
    assert n >= 0
    assert v == 0, msg


@pytest.mark.parametrize("q", [5, -5, 4, 3])
def test_quantizer_grids(lib, q):
    for name, z in GRAPHS[:4]:
        n, v, msg = bounds(lib, name, z, 20, q=q)
        assert v == 0, f"{name} q={q}: {msg}"


def test_the_survey_workloads_have_plans(lib):
    # C2 (wman), C3 (802.11n, UCN one-chunk), C4 (5G BG2, multi-chunk): several instances each
    for name, z in GRAPHS[:3]:
        n, v, _ = bounds(lib, name, z, 50)
        assert n >= 2 and v == 0, name


def test_pre_guard_read_is_caught(lib):
    """The cn_hd read without `ql < cn_lanes` (the kernel before the r4c fix): 802.11n's
    one-chunk UCN instance has 12 waves and 7 waves of check lanes, so waves 7-11 read past the
    table; the check must flag it (and the guarded read must be clean, above)."""
    n, v, msg = bounds(lib, "802_11n_N648_R56_z27", 27, 50, flags=PRE_GUARD)
    assert n > 0 and v > 0 and "cn_hd" in msg, msg
    # the graphs whose UCN instances have no waves past their check lanes stay clean
    n, v, msg = bounds(lib, "wman_N0576_R34_z24", 24, 20, flags=PRE_GUARD)
    assert v == 0, msg


def test_bsc_plan_checked(lib):
    """5G BG1 (C5) is the compressed kernel's (bsc): its plan is checked too -- the channel tables
    inside the SGN region they borrow, and every check chunk's real-position count inside the
    1 .. EPL range its min2 switch covers (the other counts are marked unreachable)."""
    name, z = GRAPHS[3]
    # (one channel weight per iteration: the uniform-lane plan and the beta = 1 mixed-lane one;
    # per-column channel tables do not fit BG1's LDS, so no kernel of the bit-sliced family
    # serves that case)
    n, v, msg = bounds(lib, name, z, 50, au=1, bu=1)
    assert n == 2 and v == 0, (n, msg)
