"""Build the native pieces in-tree (hipcc for gfx950; no JIT cache, no pip install).

Artifacts (git-ignored, shipped to the GPU box with the snapshot):
  ldpc_error_floor_amd/libldpc_nms.so          C ABI (include/ldpc_nms.h), HIP kernels
  ldpc_error_floor_amd/_ldpc_nms<EXT_SUFFIX>    pybind11 binding, rpath $ORIGIN

Usage: python -m ldpc_error_floor_amd.build [--force] [--jobs N]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(PKG, "_build")
ARCH = os.environ.get("LDPC_OFFLOAD_ARCH", "gfx950")

HIP_SOURCES = ["ldpc_capi.hip", "ldpc_flood.hip", "ldpc_fused.hip", "ldpc_fused5.hip",
               "ldpc_bs.hip", "ldpc_bsc.hip", "ldpc_ffl.hip", "ldpc_channel.hip", "ldpc_collect.hip"]
HEADERS = ["ldpc_internal.h", "ldpc_fused.h", "ldpc_fused5_kernel.h", "ldpc_bs_kernel.h", "ldpc_bitplane.h", "ldpc_awgn.h",
           "ldpc_host.h", "ldpc_quant.h"]
# host-only C++ (no HIP): also built with g++ -fsanitize=address,undefined by
# tests/test_host_sanitized.py
HOST_SOURCES = ["ldpc_host.cpp"]
# ldpc_fused5_shape.hip is compiled once per kShapes5 entry (-DF5_SHAPE=i), in parallel
F5_SHAPE_SRC = "ldpc_fused5_shape.hip"
# ldpc_bs_inst.hip is compiled once per kBsInst entry (-DBS_INST=i), in parallel
BS_INST_SRC = "ldpc_bs_inst.hip"


def _table_count(header, decl):
    import re
    src = open(os.path.join(CSRC, header)).read()
    body = src.split(decl, 1)[1].split("\n};", 1)[0]
    return len(re.findall(r"^\s*\{", body, re.M))


def _f5_shape_count():
    return _table_count("ldpc_fused5_kernel.h", "constexpr Shape5 kShapes5[] = {")


def _bs_inst_count():
    return _table_count("ldpc_bs_kernel.h", "constexpr BsInst kBsInst[] = {")
LIB = os.path.join(PKG, "libldpc_nms.so")
EXT = os.path.join(PKG, "_ldpc_nms" + sysconfig.get_config_var("EXT_SUFFIX"))


# the bit-sliced instance units (ldpc_bs_inst.hip) are scheduled with the AMDGPU register-
# pressure trackers: same box, C3 14.63 -> 14.50 ms, C4 13.74 -> 13.60, C2 unchanged; the bsc unit
# keeps the default scheduler (C5 52.3 against 52.7 ms with them; profiles/r3/ab r3zf)
BS_INST_FLAGS = ["-mllvm", "-amdgpu-use-amdgpu-trackers"]


def source_fingerprint() -> str:
    """sha256 (first 16 hex digits) of every native source and header this build compiles, plus
    the compile flags: a profile taken of one build (tools/traffic_json.py) records it, and
    bench.py uses the profile's PMC-derived figures only for the same sources."""
    import hashlib
    h = hashlib.sha256()
    files = sorted(HIP_SOURCES + HEADERS + HOST_SOURCES + [F5_SHAPE_SRC, BS_INST_SRC])
    for f in files:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(INCLUDE, "ldpc_nms.h"), "rb") as fh:
        h.update(fh.read())
    h.update(" ".join(_flags()).encode())
    h.update(" ".join(BS_INST_FLAGS).encode())
    return h.hexdigest()[:16]


def _flags(absolute=False):
    inc = (INCLUDE, CSRC) if absolute else (os.path.relpath(INCLUDE, ROOT), os.path.relpath(CSRC, ROOT))
    # the fused kernels' per-group loops must unroll completely (register-resident per-group
    # state); the default pragma threshold gives up on the wide shapes
    return ["--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
            "-I" + inc[0], "-I" + inc[1], "-Wall", "-Wno-unused-result",
            "-mllvm", "-pragma-unroll-threshold=500000"]


def _hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the HIP extension)")


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(force=False, jobs=4, verbose=False):
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "ldpc_nms.h")]
    flags = _flags(absolute=True)
    objs, jobs_list = [], []
    units = [(src, src.replace(".hip", ".o"), []) for src in HIP_SOURCES]
    units += [(src, src.replace(".cpp", ".o"), []) for src in HOST_SOURCES]
    units += [(F5_SHAPE_SRC, f"ldpc_fused5_s{i}.o", [f"-DF5_SHAPE={i}"])
              for i in range(_f5_shape_count())]
    units += [(BS_INST_SRC, f"ldpc_bs_i{i}.o", [f"-DBS_INST={i}"] + BS_INST_FLAGS)
              for i in range(_bs_inst_count())]
    for src, obj, defs in units:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, obj)
        objs.append(o)
        if force or _newer(o, [s] + hdrs + [os.path.abspath(__file__)]):   # (flags live here)
            jobs_list.append([hipcc] + flags + defs + ["-c", s, "-o", o])
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        for r in ex.map(_run, jobs_list):
            if verbose and r.stderr:
                print(r.stderr, file=sys.stderr)
    if force or _newer(LIB, objs):
        _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB] + objs)
    py_src = os.path.join(CSRC, "pybind_module.cpp")
    if force or _newer(EXT, [py_src, LIB, os.path.join(INCLUDE, "ldpc_nms.h")]):
        import pybind11
        cxx = os.environ.get("CXX", "g++")
        _run([cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-fvisibility=hidden",
              "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
              "-I" + INCLUDE, py_src, "-o", EXT, "-L" + PKG, "-lldpc_nms",
              "-Wl,-rpath,$ORIGIN"])
    return LIB, EXT


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 1))
    a = ap.parse_args()
    lib, ext = build(force=a.force, jobs=a.jobs, verbose=True)
    print(lib)
    print(ext)


if __name__ == "__main__":
    main()
