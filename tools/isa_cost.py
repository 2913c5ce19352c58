#!/usr/bin/env python3
"""Static VALU cost histogram of an ISA excerpt, priced with the gfx950 issue costs measured by
tools/valu_table.hip at 6 waves/SIMD (fast VOP1/VOP2 forms ~2.8 cycles, 32-bit min/max,
shift-left, VOP3-only, SDWA and DPP forms ~4.2, compares ~4.6).
usage: python3 tools/isa_cost.py FILE.s"""
import collections
import re
import sys

FAST32 = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_and_b32", "v_or_b32", "v_xor_b32",
          "v_lshrrev_b32", "v_ashrrev_i32", "v_mov_b32", "v_not_b32", "v_add_f32", "v_sub_f32",
          "v_subrev_f32", "v_mul_f32", "v_fmac_f32", "v_fma_f32"}


def cost(op, line):
    base = op.replace("_e32", "").replace("_e64", "")
    if "sdwa" in op or "dpp" in line:
        return 4.2
    if base in FAST32:
        return 2.8
    if re.match(r"^v_\w+_(u16|i16|b16|f16)$", base) and not base.startswith(("v_pk", "v_med3", "v_mad")):
        return 2.8
    if base.startswith(("v_cmp", "v_cndmask")) or "co_u32" in base:
        return 4.6
    return 4.2


def main():
    tot, cyc, other = collections.Counter(), collections.Counter(), collections.Counter()
    for l in open(sys.argv[1]):
        t = l.strip()
        if not t or t[0] in ";.":
            continue
        op = t.split()[0]
        if not op.startswith("v_"):
            other[op] += 1
            continue
        if "sdwa" in t:
            op += "(sdwa)"
        tot[op] += 1
        cyc[op] += cost(op, t)
    print(sum(tot.values()), "VALU, est. cycles", round(sum(cyc.values())))
    for op, c in cyc.most_common(60):
        print(f"{op:28s} {tot[op]:5d} {c:8.0f}")
    print(other.most_common(25))


if __name__ == "__main__":
    main()
