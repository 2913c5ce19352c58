"""The bit-sliced kernels' plane arithmetic on the host (CPU only): csrc/ldpc_bitplane.h is
HIP-free, so tests/native/bitplane_check.cpp includes it with v_bitop3_b32 emulated from its truth
table and checks every function the variable and check phases build on, exhaustively over the
ranges the kernels use -- the C->V sums of set_b / add_b at 7, 8 and 9 planes, clamp6, V->C =
clamp(Tv - m, +-15) as sign and magnitude by sub_tv + abs_sat (Main_Functions.py:213-230), and
lt4 -- for the default build and for the earlier forms kept behind -DBS_SETB=0."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "ldpc_error_floor_amd", "csrc")
SRC = os.path.join(ROOT, "tests", "native", "bitplane_check.cpp")


@pytest.mark.parametrize("defs", [[], ["-DBS_SETB=0", "-DBS_ABS12=0"], ["-DBS_SETB_SIGN=1"]])
def test_plane_arithmetic_exhaustive(tmp_path, defs):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "bitplane_check")
    subprocess.run([cxx, "-O2", "-std=c++17", "-I" + CSRC] + defs + [SRC, "-o", exe], check=True,
                   capture_output=True, text=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    assert r.stdout.startswith("ok ")
