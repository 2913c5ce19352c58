"""SURVEY.md §5 "race detection / sanitizers": the host-only half of the C ABI
(csrc/ldpc_host.cpp — graph tables, weight analysis, argument validation; the same code
libldpc_nms.so runs before touching the device) built with g++ -fsanitize=address,undefined
and driven by tests/native/host_check.cpp: the argument-validation cases of the ABI,
3000 randomized proto matrices / weight tables, and the tables of every shipped base graph,
which must equal the Python TannerGraph's (CPU only).

(This check found an out-of-bounds read in the row-merge analysis for an all -1 proto row.)"""
import glob
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT
from ldpc_error_floor_amd.code import TannerGraph, load_base_graph

CSRC = os.path.join(ROOT, "ldpc_error_floor_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]
ZS = {"wman_N0576_R34_z24": 24, "802_11n_N648_R56_z27": 27, "MACKAY_N96_K48": 1,
      "BCH_63_51": 1, "Polar_64_48": 1}


@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("asan") / "host_check")
    subprocess.run([cxx, "-std=c++17", "-O1", "-g"] + SAN +
                   ["-I" + os.path.join(ROOT, "include"), "-I" + CSRC,
                    os.path.join(CSRC, "ldpc_host.cpp"),
                    os.path.join(ROOT, "tests", "native", "host_check.cpp"), "-o", exe],
                   check=True, capture_output=True, text=True)
    return exe


def _run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    return subprocess.run([exe, *args], capture_output=True, text=True, env=env, timeout=300)


def test_validation_and_fuzz_under_sanitizers(host_check):
    r = _run(host_check, "selftest", "3000")
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "0 failures" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(
    ROOT, "ldpc_error_floor_amd", "data", "BaseGraph", "*.txt"))), ids=os.path.basename)
def test_tables_equal_python_graph(host_check, path):
    name = os.path.basename(path)[:-4]
    z = ZS.get(name) or int(name.split("_z")[1].split("_")[0])
    r = _run(host_check, "tables", path, str(z))
    assert r.returncode == 0, r.stderr[-4000:]
    t = json.loads(r.stdout)
    g = TannerGraph(load_base_graph(path), z)
    if g.max_check_deg > 64:
        assert t["status"] == -5
        return
    assert t["status"] == 0 and (t["M"], t["N"], t["E"]) == (g.M, g.N, g.E)
    assert t["max_cdeg"] == g.max_check_deg and t["max_vdeg"] == g.max_var_deg
    np.testing.assert_array_equal(t["row_ptr"], g.row_ptr)
    np.testing.assert_array_equal(t["pe_col"], g.pe_col)
    np.testing.assert_array_equal(t["pe_shift"], g.pe_shift)
    col_ptr = np.concatenate([[0], np.cumsum(g.vn_deg)])
    np.testing.assert_array_equal(t["col_ptr"], col_ptr)
    np.testing.assert_array_equal(np.asarray(t["col_pe"]), np.lexsort((g.pe_row, g.pe_col)))


@pytest.mark.parametrize("q", [6, 5, -5, 4, 3])
@pytest.mark.parametrize("sigma", [0.4, 0.5478, 0.61, 0.7943282, 1.1])
def test_qms_thresholds_equal_oracle(host_check, q, sigma):
    """The channel's level-sampler tables (host::awgn_qms_levels: erfc in float64, the 64-bit
    CDF threshold of each rounding boundary) equal the oracle's restatement bit for bit — what
    the GPU sampler compares its Philox words against (tests/test_gpu_channel.py checks the
    levels it draws)."""
    from oracle.philox_oracle import qms_levels
    r = _run(host_check, "qms", repr(sigma), str(q))
    assert r.returncode == 0, r.stderr[-2000:]
    t = json.loads(r.stdout)
    T, vals, kmin = qms_levels(sigma, q)
    assert t["nb"] == len(T) and t["kmin"] == kmin
    assert [int(x) for x in t["thr"]] == [int(x) for x in T]
    np.testing.assert_array_equal(np.float32(t["val"]), vals)
