#!/usr/bin/env python3
"""Per-basic-block instruction mix of one kernel in a hipcc --save-temps .s file.
usage: python3 tools/isa_blocks.py FILE.s SYMBOL_SUBSTRING"""
import re
import sys

src, want = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*:", l) and want in l)
blocks, cur = [], None
for l in lines[start:]:
    m = re.match(r"^(\.LBB\w+|_Z\w+):", l)
    if m:
        cur = [m.group(1), 0, 0, 0, 0, []]
        blocks.append(cur)
        continue
    s = l.strip()
    if not s or s.startswith(";") or s.startswith("."):
        continue
    op = s.split()[0]
    if op.startswith("v_"):
        cur[1] += 1
    elif op.startswith(("s_waitcnt", "s_barrier", "s_nop")):
        cur[4] += 1
    elif op.startswith("s_"):
        cur[2] += 1
    elif op.startswith("ds_"):
        cur[3] += 1
    if op.startswith(("s_cbranch", "s_branch")):
        cur[5].append(s.split()[0][9:] + ":" + s.split()[-1])
    if op == "s_endpgm":
        break
for b in blocks:
    print(f"{b[0][:28]:28s} V{b[1]:4d} S{b[2]:4d} DS{b[3]:3d} W{b[4]:3d} {' '.join(b[5])[:80]}")
