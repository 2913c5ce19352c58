#!/usr/bin/env python3
"""Copy one tools/evidence.sh run (gpurun_out/ev_<TAG>) into the tracked profiles/ tree:
per-config kernel stats + PMC summaries, the bench line, the rocprofv3 kernel-trace summary of
the bench command, and profiles/traffic_<kernel>.json (read by bench.py) with its "source"
pointing at the committed copy.
usage: python3 tools/collect_evidence.py gpurun_out/ev_c profiles/r2/c"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for cfg in sorted(glob.glob(os.path.join(src, "C*"))):
        if os.path.isdir(cfg):
            shutil.copytree(cfg, os.path.join(dst, os.path.basename(cfg)), dirs_exist_ok=True)
    for f in ("bench_c2.json", "bench_c2_traced.json"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), dst)
    ks = os.path.join(src, "bench_trace", "bench_kernel_stats.csv")
    if os.path.exists(ks):
        shutil.copy(ks, os.path.join(dst, "bench_c2_rocprof_kernel_stats.csv"))
    sys.path.insert(0, ROOT)
    from ldpc_error_floor_amd.build import source_fingerprint
    fp = source_fingerprint()
    for tj in glob.glob(os.path.join(src, "traffic_fused5_*.json")) + \
            glob.glob(os.path.join(src, "traffic_bsl_*.json")) + \
            glob.glob(os.path.join(src, "traffic_bsc_*.json")) + \
            glob.glob(os.path.join(src, "traffic_flood*.json")):
        d = json.load(open(tj))
        if d.get("src_fingerprint") != fp:       # another build's profile that rode along
            continue
        old = d.get("source", "")
        cfg = os.path.basename(old.rstrip("/"))
        d["source"] = os.path.relpath(os.path.join(dst, cfg), ROOT)
        with open(os.path.join(ROOT, "profiles", os.path.basename(tj)), "w") as f:
            json.dump(d, f, indent=1)
        shutil.copy(os.path.join(ROOT, "profiles", os.path.basename(tj)), dst)
    print("collected", src, "->", dst)


if __name__ == "__main__":
    main()
