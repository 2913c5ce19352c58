#!/usr/bin/env python3
"""The two-kernel (north-star) flood decoder against the HBM roofline, per kernel: from a
tools/profile.sh directory of `K=flood` (kernel trace + FETCH_SIZE / WRITE_SIZE passes).

    python3 tools/flood_roofline.py gpurun_out/prof_<TAG>_C2_flood --batch 1048576 \\
        --out profiles/r4/flood

For the steady-state launches of k_cn_update (t > 0) and k_vn_update (t < T - 1) it reports
the average duration (rocprofv3 trace), the design bytes per codeword of that launch (the
SURVEY §8 d model restricted to the kernel: CN reads Tv and C->V, writes C->V; VN reads C->V
and the channel, writes Tv and the hard bits), achieved = design bytes x B / duration, the
measured HBM bytes per launch (FETCH_SIZE doubled, + WRITE_SIZE, KiB: MI355X_MICROARCH.md HBM
section), and both against 8 TB/s.  Writes <out>/flood_roofline.json and copies the trace
summary."""
import argparse
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HBM_PEAK = 8.0e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    import bench
    cfg = bench.CONFIGS[a.config]
    proto, g, W, cp = bench.load_problem(config=a.config)
    nv, ne = g.N * cfg["z"], g.E * cfg["z"]
    design = {"k_cn_update": 4 * nv + 4 * ne + 4 * ne,           # Tv, C->V in; C->V out
              "k_vn_update": 4 * ne + 4 * nv + 4 * nv + nv // 8}  # C->V, ch in; Tv, hd out
    stats = {}
    for f in glob.glob(os.path.join(a.prof, "trace", "*kernel_stats.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                stats[row["Name"]] = (float(row["AverageNs"]), int(row["Calls"]))
        os.makedirs(a.out, exist_ok=True)
        shutil.copy(f, os.path.join(a.out, "flood_kernel_stats.csv"))
    pmc = {}
    for f in sorted(glob.glob(os.path.join(a.prof, "pmc*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                pmc.setdefault((row["Kernel_Name"], row["Counter_Name"]), []).append(float(row["Counter_Value"]))
    out = {"config": a.config, "batch": a.batch, "peak_bytes_per_s": HBM_PEAK, "kernels": {}}
    for kname, (avg, calls) in stats.items():
        short = next((k for k in design if k in kname), None)
        # the steady-state builds: k_cn_update<MODE, FIRST=false, UCN>, k_vn_update<MODE, LAST=false>
        if short is None or kname.split("<", 1)[1].split(",", 2)[1].strip().startswith("true"):
            continue
        bpc = design[short]
        ach = bpc * a.batch / (avg * 1e-9)
        ent = {"name": kname, "calls": calls, "avg_ns": round(avg), "design_bytes_per_cw": bpc,
               "achieved_GBps": round(ach / 1e9, 1), "achieved_frac": round(ach / HBM_PEAK, 4)}
        fs = pmc.get((kname, "FETCH_SIZE"))
        ws = pmc.get((kname, "WRITE_SIZE"))
        if fs and ws:
            traffic = 2.0 * 1024.0 * sum(fs) / len(fs) + 1024.0 * sum(ws) / len(ws)
            ent.update({"hbm_bytes_per_launch": round(traffic),
                        "hbm_bytes_per_cw": round(traffic / a.batch, 1),
                        "measured_GBps": round(traffic / (avg * 1e-9) / 1e9, 1),
                        "measured_frac": round(traffic / (avg * 1e-9) / HBM_PEAK, 4)})
        out["kernels"][short] = ent
    os.makedirs(a.out, exist_ok=True)
    with open(os.path.join(a.out, "flood_roofline.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
