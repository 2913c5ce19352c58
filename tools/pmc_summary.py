#!/usr/bin/env python3
"""Summarise rocprofv3 PMC csv passes per kernel: mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    vals = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"]
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return vals


def durations(d):
    out = {}
    for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                out[row["Name"]] = float(row["AverageNs"])
    return out


if __name__ == "__main__":
    d = sys.argv[1]
    dur = durations(d)
    for k, cs in load(d).items():
        if "ldpc" not in k:
            continue
        short = k.split("(")[0]
        print(f"== {short}  avg {dur.get(k, float('nan'))/1e3:.1f} us")
        for c, v in sorted(cs.items()):
            print(f"   {c:24s} {sum(v)/len(v):16.4g}  (n={len(v)})")
