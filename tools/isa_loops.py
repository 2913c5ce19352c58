#!/usr/bin/env python3
"""Outermost loops of a kernel's ISA (the compiler's own "Loop Header: Depth=1" annotations) and
what their bodies hold: VALU ops, SGPR-spill lane moves (v_writelane / v_readlane), scratch
accesses, LDS / scalar-memory ops, barriers.

    python3 tools/isa_loops.py FILE.s [kernel-substring]

Static counts over the text of each depth-1 loop (the blocks annotated as its members and the
nested loops between them): enough to see whether spill code or reloads sit inside the
T-iteration loop (the depth-1 loop with the barriers)."""
import re
import sys


def main():
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    lines = open(path).read().splitlines()
    funcs, cur, start = [], None, 0
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur, start = m.group(1), i
        elif cur and l.startswith(".Lfunc_end"):
            funcs.append((cur, start, i))
            cur = None
    for name, a, b in funcs:
        if want and want not in name:
            continue
        first, last = {}, {}
        for i in range(a, b):
            m = re.match(r"^\.(LBB\S+):\s*;.*(?:Loop Header|in Loop: Header=(BB\S+)) ?.*Depth=1", lines[i])
            if not m:
                continue
            h = m.group(2) or m.group(1)[1:]
            first.setdefault(h, i)
            last[h] = i
        print(name[:110], f"lines {b - a}")
        for h in first:
            s = first[h]
            e = last[h]
            while e + 1 < b and not re.match(r"^\.LBB\S+:", lines[e + 1]):   # end of the last block
                e += 1
            ops = [x.strip().split()[0] for x in lines[s:e + 1]
                   if x.strip() and not x.strip().startswith((";", ".")) and not x.strip().endswith(":")]
            c = lambda p: sum(1 for o in ops if o.startswith(p))   # noqa: E731
            print(f"  loop {h} lines {s}-{e}: ops {len(ops)} VALU {c('v_')} writelane {c('v_writelane')} "
                  f"readlane {c('v_readlane')} scratch {c('scratch_')} ds {c('ds_')} smem {c('s_load')} "
                  f"vmem {c('global_') + c('buffer_')} barrier {c('s_barrier')} waitcnt {c('s_waitcnt')}")


if __name__ == "__main__":
    main()
