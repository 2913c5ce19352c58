#!/usr/bin/env python3
"""Turn a tools/profile.sh output directory into the files committed under profiles/.

  python3 tools/traffic_json.py gpurun_out/prof_<TAG>_<K> --batch 1048576 --out profiles/r1

Writes
  <out>/<kernel>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  <out>/<kernel>_pmc.txt            per-dispatch means of every PMC counter collected
  profiles/traffic_<kernel>.json    {"batch", "hbm_bytes_per_launch", ...} read by bench.py

HBM bytes follow MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB and
come from separate --pmc passes; on gfx950 FETCH_SIZE counts half the bytes of a coalesced
read, so it is doubled; WRITE_SIZE is taken as is.  <kernel> is the decoder's display name
(ldpc_kernel_info) with characters outside [A-Za-z0-9_.-] replaced by '_'.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def safe_name(name):
    return re.sub(r"[^A-Za-z0-9_.-]", "_", name)


def dominant_kernel(prof):
    """(mangled-ish name, average ns) of the longest ldpc kernel other than the AWGN generator."""
    best = None
    for f in glob.glob(os.path.join(prof, "trace", "*kernel_stats.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                n = row["Name"]
                if "ldpc" not in n or "k_awgn" in n:
                    continue
                avg = float(row["AverageNs"])
                if best is None or avg > best[1]:
                    best = (n, avg, int(row["Calls"]))
    return best


def pmc_means(prof, kernel):
    vals = {}
    for f in sorted(glob.glob(os.path.join(prof, "pmc*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Kernel_Name"] != kernel:
                    continue
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def valu_busy(pm, avg_ns):
    """Fraction of the SIMDs' VALU issue time in use.  A SIMD-32 issues a wave64 VALU
    instruction over 2 cycles, so a quad-cycle holds one or two VALU issues (two only for
    instructions that fit 2 cycles; VOP3/SDWA forms take the whole quad-cycle,
    DESIGN.md 3.2): busy quad-cycles = SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2 (the quad-cycles
    with two).  Available quad-cycles = 1024 SIMDs x (GRBM_GUI_ACTIVE / 8 XCDs) / 4."""
    need = ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU2", "GRBM_GUI_ACTIVE")
    if not all(k in pm for k in need):
        return None
    busy = pm["SQ_INSTS_VALU"] - pm["SQ_ACTIVE_INST_VALU2"]
    avail = 1024 * (pm["GRBM_GUI_ACTIVE"] / 8.0) / 4.0
    return {"frac": round(busy / avail, 4), "busy_quad_cycles": round(busy),
            "dual_issue_quad_cycles": round(pm["SQ_ACTIVE_INST_VALU2"]),
            "clock_ghz": round(pm["GRBM_GUI_ACTIVE"] / 8.0 / avg_ns, 3)}


def lds_busy(pm):
    """Fraction of the CUs' LDS-array cycles in use: SQ_LDS_IDX_ACTIVE (LDS-array cycles summed
    over the 256 CUs, bank-conflict cycles included: SQ_LDS_BANK_CONFLICT) over 256 x
    (GRBM_GUI_ACTIVE / 8 XCDs) (MI355X_MICROARCH.md, LDS)."""
    if "SQ_LDS_IDX_ACTIVE" not in pm or "GRBM_COUNT" not in pm:
        return None
    avail = 256 * pm["GRBM_COUNT"] / 8.0
    out = {"frac": round(pm["SQ_LDS_IDX_ACTIVE"] / avail, 4)}
    if "SQ_LDS_BANK_CONFLICT" in pm:
        out["conflict_frac"] = round(pm["SQ_LDS_BANK_CONFLICT"] / pm["SQ_LDS_IDX_ACTIVE"], 4)
    return out


def display_name(prof):
    with open(os.path.join(prof, "trace.log")) as fh:
        for line in fh:
            m = re.search(r"kernel (\S+)\s*$", line)
            if m:
                return m.group(1)
    raise SystemExit("no 'kernel <name>' line in trace.log")


def src_fingerprint():
    """The native sources' fingerprint (ldpc_error_floor_amd.build.source_fingerprint): bench.py
    uses this profile's PMC figures only while the sources are unchanged."""
    sys.path.insert(0, ROOT)
    from ldpc_error_floor_amd.build import source_fingerprint
    return source_fingerprint()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof")
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--source", default=None,
                    help="path recorded as the profile's home (default: --out), e.g. the "
                         "profiles/<round>/... directory the files are committed under")
    a = ap.parse_args()
    dk = dominant_kernel(a.prof)
    if dk is None:
        raise SystemExit("no ldpc kernel in the trace")
    kernel, avg_ns, calls = dk
    name = display_name(a.prof)
    sn = safe_name(name)
    os.makedirs(a.out, exist_ok=True)
    for f in glob.glob(os.path.join(a.prof, "trace", "*kernel_stats.csv")):
        shutil.copy(f, os.path.join(a.out, f"{sn}_kernel_stats.csv"))
    pm = pmc_means(a.prof, kernel)
    with open(os.path.join(a.out, f"{sn}_pmc.txt"), "w") as fh:
        fh.write(f"# {kernel}\n# display name {name}, batch {a.batch}, trace average "
                 f"{avg_ns / 1e3:.1f} us over {calls} calls\n")
        for k in sorted(pm):
            fh.write(f"{k:24s} {pm[k]:.6g}\n")
    if "FETCH_SIZE" not in pm or "WRITE_SIZE" not in pm:
        print("FETCH_SIZE/WRITE_SIZE missing: traffic not written", file=sys.stderr)
        return
    fetch = 2.0 * pm["FETCH_SIZE"] * 1024.0
    write = pm["WRITE_SIZE"] * 1024.0
    tj = {"kernel": name, "batch": a.batch, "hbm_bytes_per_launch": round(fetch + write),
          "fetch_bytes": round(fetch), "write_bytes": round(write),
          "bytes_per_codeword": round((fetch + write) / a.batch, 1),
          "avg_launch_ns": round(avg_ns), "source": a.source or os.path.relpath(a.out, ROOT),
          "valu_insts_per_launch": round(pm["SQ_INSTS_VALU"]) if "SQ_INSTS_VALU" in pm else None,
          "wait_any_frac": (round(pm["SQ_WAIT_ANY"] / pm["SQ_WAVE_CYCLES"], 4)
                            if "SQ_WAIT_ANY" in pm and pm.get("SQ_WAVE_CYCLES") else None),
          "valu_busy": valu_busy(pm, avg_ns),
          "src_fingerprint": src_fingerprint(),
          "lds_busy": lds_busy(pm),
          "method": "2 x FETCH_SIZE + WRITE_SIZE (KiB), separate --pmc passes, gfx950 "
                    "FETCH_SIZE half-count correction (MI355X_MICROARCH.md, HBM)"}
    path = os.path.join(ROOT, "profiles", f"traffic_{sn}.json")
    with open(path, "w") as fh:
        json.dump(tj, fh, indent=1)
    print(json.dumps(tj))


if __name__ == "__main__":
    main()
