#!/usr/bin/env python3
"""Per-phase VALU attribution of a bit-sliced kernel's T loop, by instruction form.

    python3 tools/isa_phase_table.py FILE.s KERNEL-SUBSTRING --dw 6,6,6,3,3,3,3,3,2 \
        --cwaves 9 --edges 2112 [--json OUT]

FILE.s is a `-DBS_MARK` build of one kernel instance (hipcc --cuda-device-only -S): the kernel
then carries ";@ph NAME.K" assembler comments at each phase start (ldpc_bs_kernel.h, PH()).
The tool takes the depth-1 loop that holds the barriers (the T loop), builds its control-flow
graph, gives every basic block the phase of the marker last seen on the way into it (so the
compiler's out-of-line blocks, e.g. pass 2 placed after the variable phase, keep their phase),
and counts each VALU instruction by form, with the issue cost measured by tools/valu_rate.hip on
gfx950 (profiles/r5/valu_rate.log, 8 waves per SIMD):

  v2   VOP1 / VOP2 / VOP3 forms with VGPR or inline-constant operands: ~2.3-2.5 cycles
       (v_bitop3_b32, v_xor / v_and / v_or, v_add_u32, v_lshrrev, v_not, v_mov)
  sgpr a VOP1/2/3 with an SGPR (or VCC / EXEC) operand: ~4.1-4.3 cycles
  dpp  a DPP form (v_mov_b32_dpp, v_xor_b32_dpp, ...): ~4.1-4.2 cycles
  sdwa an SDWA form: ~4.1 cycles
  slow v_min / v_max / v_med3 / v_perm / v_alignbit / v_add3 / v_pk_* / v_mul* / v_mad*: ~4.1
  lane v_readlane / v_writelane / v_readfirstlane (spill and reduction traffic)

Counts are static (one pass over each block), then weighted per pack-iteration: the check
phases by the check waves (--cwaves), the per-variable phases by the variable waves (the length
of --dw), and the per-edge phases (vn_sum.f, vn_vc.f) by the waves whose largest variable degree
exceeds f (--dw: each wave's most edges of a variable).  The ";@ph" markers are scheduling
boundaries, so the marked build's totals are compared with the product build's (--product):
the split is the marked build's, the totals of both are printed.  The last iteration's copy of
the variable phase (markers K >= 100) is reported separately; the table is one non-last
iteration, i.e. per pack-edge-iteration for T >> 1.

  --sbv MAX,SET   the plane-count copies of the variable phase (BS_SBV: markers carry
                  1000 (planes - 6)) weighted by the places that run each: MAX the instance's
                  planes of S, SET its BS_SBV_SET (1 seven, 2 eight)
  --mc NW,VPL,CPL --vchunks D,... --cchunks G,...
                  multi-chunk instances: the host's dealing of the variable chunks (largest
                  degree each) and check chunks (real positions each) to (wave, place) slots is
                  replayed (deal_chunks), and each marker is weighted by the slots that run it
                  (check markers K = 16 c + position, variable markers K = 10 u + edge)
  --dump P,...    the static VALU mnemonics of these phases (where the forms come from)

    python3 tools/isa_phase_table.py c4.s Li4ELb0ELi1024ELb0E --dw 1 --cwaves 1 --edges 4288 \
        --mc 16,2,2 --vchunks 8,7,7,5,5,4,4,4,3,3,3,3,3,2,1,1,1,1,1,1 \
        --cchunks 4,4,5,5,4,4,5,5,2,2,3,3,3,3,3,3,2,2,3,3 --sbv 9,2
"""
import argparse
import json
import re
import sys
from collections import defaultdict

SLOW = re.compile(r"^v_(min|max|med3|perm|alignbit|add3|pk_|mul|mad|sad|cvt|lshl_add|lshl_or|and_or|or3|xad|"
                  r"bfe|bfi|alignbyte|cndmask_b32_e64|subrev_co|add_co|sub_co|ldexp|frexp|exp|log|rcp|rsq|sqrt|sin|cos)")
TWO = re.compile(r"^v_(bitop3|xor|and|or|not|xnor|add_u32|sub_u32|subrev_u32|lshrrev|lshlrev|ashrrev|mov_b32|"
                 r"bfrev|cndmask_b32_e32)")
SREG = re.compile(r"(?<![\w])(s\d+|s\[\d+:\d+\]|vcc|vcc_lo|vcc_hi|exec|exec_lo|exec_hi|m0|ttmp\d+)(?![\w])")


def classify(ins):
    op = ins.split()[0]
    if not op.startswith("v_"):
        return None
    if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
        return "lane"
    if "_dpp" in op or " quad_perm" in ins or "row_" in ins:
        return "dpp"
    if "_sdwa" in op or "dst_sel" in ins:
        return "sdwa"
    operands = ins[len(op):]
    # (v_cndmask_b32_e32 reads VCC implicitly; the e64 form names its SGPR pair)
    if SREG.search(operands) or op.startswith("v_cndmask_b32_e32"):
        return "sgpr"
    if SLOW.match(op):
        return "slow"
    return "v2"


COST = {"v2": 2.4, "sgpr": 4.2, "dpp": 4.2, "sdwa": 4.1, "slow": 4.1, "lane": 4.3}
FORMS = ["v2", "sgpr", "dpp", "sdwa", "slow", "lane"]


def function_lines(lines, want):
    cur, start = None, 0
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\S+):", l)
        if m:
            cur, start = m.group(1), i
        elif cur and l.startswith(".Lfunc_end"):
            if want in cur:
                return cur, lines[start:i]
            cur = None
    raise SystemExit(f"no kernel matching {want!r}")


def blocks_of(body):
    """[(name, [lines])]: a block starts at a label or a '; %bb.N:' comment"""
    blocks, name, cur = [], "entry", []
    for l in body:
        m = re.match(r"^(\.L\w+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), [l]
        else:
            cur.append(l)
    blocks.append((name, cur))
    return blocks


def insts(lines):
    for l in lines:
        t = l.strip()
        if t.startswith(";@ph"):
            yield ("mark", t.split()[1])
        elif t and not t.startswith((";", ".")) and not t.endswith(":"):
            yield ("ins", t.split(";")[0].strip())


def analyse(path, want):
    lines = open(path).read().splitlines()
    name, body = function_lines(lines, want)
    blocks = blocks_of(body)
    idx = {b[0]: i for i, b in enumerate(blocks)}
    # the T loop: the depth-1 loop whose blocks hold s_barrier
    hdr_of = {}
    for bn, bl in blocks:
        head = bl[0] if bl else ""
        m = re.search(r"Loop Header: Depth=1", head)
        if m:
            hdr_of[bn] = bn.lstrip(".L")
        m = re.search(r"(?:in Loop: Header|Parent Loop) (?:=)?(BB\w+)", head) or re.search(r"Header=(BB\w+) Depth=1", head)
        if m:
            hdr_of[bn] = m.group(1)
    loops = defaultdict(list)
    for bn, h in hdr_of.items():
        loops[h].append(bn)
    tloop = None
    for h, bns in loops.items():
        if any("s_barrier" in l for bn in bns for l in blocks[idx[bn]][1]):
            tloop = h
    if tloop is None:
        raise SystemExit("no loop with barriers")
    members = set(loops[tloop])
    # table regions (.LbtabN .. .LbendN): jumped into by s_swappc, one entry per call
    tables = {}
    for bn, bl in blocks:
        if bn.startswith(".Lbtab"):
            k = bn[len(".Lbtab"):]
            j = idx[bn]
            region = []
            while j < len(blocks) and blocks[j][0] != ".Lbend" + k:
                region += list(insts(blocks[j][1]))
                j += 1
            entries = max(1, sum(1 for kind, x in region if kind == "ins" and x.startswith("s_setpc")))
            valu = [classify(x) for kind, x in region if kind == "ins" and classify(x)]
            tables[k] = (entries, valu)
    table_blocks = set()
    for bn, bl in blocks:
        if bn.startswith(".Lbtab"):
            j = idx[bn]
            k = bn[len(".Lbtab"):]
            while j < len(blocks) and blocks[j][0] != ".Lbend" + k:
                table_blocks.add(blocks[j][0])
                j += 1
    # CFG successors
    def succs(i):
        bn, bl = blocks[i]
        ins = [x for kind, x in insts(bl) if kind == "ins"]
        last = ins[-1] if ins else ""
        out = []
        m = re.match(r"s_(c?branch)\w*\s+(\.L\w+)", last)
        if m:
            out.append(m.group(2))
            if m.group(1) == "cbranch" and i + 1 < len(blocks):
                out.append(blocks[i + 1][0])
        elif not last.startswith(("s_endpgm", "s_setpc")) and i + 1 < len(blocks):
            out.append(blocks[i + 1][0])
        return out
    # phase propagation from the loop header (breadth first, first arrival wins)
    head = "." + "L" + tloop if ("." + "L" + tloop) in idx else None
    if head is None:
        head = [bn for bn in members if bn.endswith(tloop)][0]
    entry_phase = {head: "top.0"}
    order = [head]
    counts = defaultdict(lambda: defaultdict(int))   # phase -> form -> static count
    other = defaultdict(lambda: defaultdict(int))    # phase -> kind (lds, salu, ...)
    seen = set()
    while order:
        bn = order.pop(0)
        if bn in seen:
            continue
        seen.add(bn)
        ph = entry_phase[bn]
        i = idx[bn]
        for kind, x in insts(blocks[i][1]):
            if kind == "mark":
                ph = x
                continue
            c = classify(x)
            if c:
                counts[ph][c] += 1
                DUMP[ph.rsplit(".", 1)[0]][x.split()[0] + ("/" + c if c != "v2" else "")] += 1
            elif x.startswith("ds_"):
                other[ph]["lds"] += 1
            elif x.startswith("s_swappc"):
                # the call into a table: count one entry's average VALU here
                k = re.search(r"\.Lbtab(\w+)", " ".join(blocks[i][1]))
                for kk, (entries, valu) in tables.items():
                    if ("Lbtab" + kk) in " ".join(blocks[i][1]) or not k:
                        for f in valu:
                            counts[ph][f] += 1.0 / entries
                        other[ph]["table_calls"] += 1
                        break
            elif x.startswith("s_") and not x.startswith(("s_waitcnt", "s_nop", "s_barrier")):
                other[ph]["salu"] += 1
        for s in succs(i):
            if s in members and s not in seen and s not in table_blocks:
                entry_phase.setdefault(s, ph)
                order.append(s)
    return name, counts, other, tables


DUMP = defaultdict(lambda: defaultdict(int))   # phase -> mnemonic/form -> static count (--dump)


def deal_chunks(cost, nw, cap):
    """ldpc_bs.hip deal_chunks (LPT): slot[w * cap + u] = chunk or -1"""
    n = len(cost)
    order = sorted(range(n), key=lambda c: -cost[c])
    vch, vload = [[] for _ in range(nw)], [0] * nw
    for c in order:
        best = -1
        for w in range(nw):
            if len(vch[w]) < cap and (best < 0 or vload[w] < vload[best] or
                                      (vload[w] == vload[best] and len(vch[w]) < len(vch[best]))):
                best = w
        vch[best].append(c)
        vload[best] += cost[c]
    vorder = sorted(range(nw), key=lambda w: -vload[w])
    sload, nxt = [0] * 4, list(range(4))
    slot = [-1] * (nw * cap)
    for v in vorder:
        sm = -1
        for q in range(4):
            if nxt[q] < nw and (sm < 0 or sload[q] < sload[sm]):
                sm = q
        w = nxt[sm]
        nxt[sm] += 4
        sload[sm] += vload[v]
        for u, c in enumerate(vch[v]):
            slot[w * cap + u] = c
    return slot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--dw", required=True, help="per variable wave: its largest variable degree")
    ap.add_argument("--cwaves", type=float, required=True, help="waves holding check lanes")
    ap.add_argument("--edges", type=int, required=True, help="lifted edges")
    ap.add_argument("--product", help="the product (unmarked) build's .s, for the totals")
    ap.add_argument("--alt", default="vn_beta_fix=1,vn_beta_id=0,vn_beta_sg=0,vn_beta_lds=0",
                    help="weights of the alternative paths (the share of iterations taking each)")
    ap.add_argument("--mc", help="multi-chunk instances: NW,VPL,CPL; with --vchunks / --cchunks the "
                    "weights come from the host's dealing of the chunks to (wave, place) slots")
    ap.add_argument("--vchunks", help="--mc: each variable chunk's largest degree, in chunk order")
    ap.add_argument("--cchunks", help="--mc: each check chunk's real edge positions per lane (gm)")
    ap.add_argument("--sbv", help="MAX,SET: the instance's planes of S and its BS_SBV_SET (the "
                    "plane-count copies' markers carry 1000 (planes - 6))")
    ap.add_argument("--dump", help="print the static VALU mnemonics of these phases (comma list)")
    ap.add_argument("--json")
    a = ap.parse_args()
    alt = {kv.split("=")[0]: float(kv.split("=")[1]) for kv in a.alt.split(",") if kv}
    dw = [int(x) for x in a.dw.split(",")]
    name, counts, other, tables = analyse(a.asm, a.kernel)
    mc = None
    if a.mc:
        nw, vpl, cpl = (int(x) for x in a.mc.split(","))
        vd = [int(x) for x in a.vchunks.split(",")]
        cg = [int(x) for x in a.cchunks.split(",")]
        vs, cs = deal_chunks([3 + d for d in vd], nw, vpl), deal_chunks([2 + g for g in cg], nw, cpl)
        # places[u] = degrees of the chunks at place u; cplaces[c] = gm of the chunks at place c
        places = [[vd[vs[w * vpl + u]] for w in range(nw) if vs[w * vpl + u] >= 0] for u in range(vpl)]
        cplaces = [[cg[cs[w * cpl + c]] for w in range(nw) if cs[w * cpl + c] >= 0] for c in range(cpl)]
        mc = (nw, places, cplaces)

    def planes(d):        # the variable-phase copy a place of largest degree d runs (BS_SBV)
        if not a.sbv:
            return None
        smax, sset = (int(x) for x in a.sbv.split(","))
        if (sset & 1) and 15 * d + 15 <= 63:
            return 7
        if (sset & 2) and smax == 9 and 15 * d + 15 <= 127:
            return 8
        return smax

    def weight(ph):
        base, k = ph.rsplit(".", 1)
        k = int(k, 0)
        sb = 6 + k // 1000 if k >= 1000 else None    # the plane-count copy of the variable phase
        k %= 1000
        last = k >= 100
        k %= 100
        w = weight1(base, k, last)
        if sb is None or not a.sbv:
            return w
        # only the places that run this copy
        if mc:
            nw, places, cplaces = mc
            u = k // 10 if base in ("vn_sum", "vn_vc") else k
            f = k % 10 if base in ("vn_sum", "vn_vc") else -1
            n = sum(1 for d in places[u] if planes(d) == sb and d > f)
        else:
            f = k if base in ("vn_sum", "vn_vc") else -1
            n = sum(1 for d in dw if planes(d) == sb and d > f)
        if base in alt:
            n *= alt[base]
        return w[0], w[1], n

    def weight1(base, k, last):
        if mc:
            nw, places, cplaces = mc
            if base == "ck_mink":
                return "ck_min", last, sum(1 for g in cplaces[k // 16] if g == k % 16)
            if base == "ck_pass2":            # K = 16 c + position m
                return base, last, sum(1 for g in cplaces[k // 16] if g > k % 16)
            if base.startswith("ck_"):
                return base, last, len(cplaces[k])
            if base in ("vn_sum", "vn_vc"):
                return base, last, sum(1 for d in places[k // 10] if d > k % 10)
            if base in alt:
                return "vn_beta", last, alt[base] * len(places[k])
            if base.startswith("vn_") and base != "vn_flags":
                return base, last, len(places[k])
            return base, last, nw
        if base in alt:
            return "vn_beta", last, alt[base] * len(dw)
        if base.startswith(("ck_", "top")):
            return base, last, a.cwaves if base.startswith("ck_") else len(dw)
        if base in ("vn_sum", "vn_vc"):
            return base, last, sum(1 for d in dw if d > k)
        return base, last, len(dw)

    rows = defaultdict(lambda: defaultdict(float))
    rows_last = defaultdict(lambda: defaultdict(float))
    for ph, fc in counts.items():
        base, last, w = weight(ph)
        tgt = rows_last if last else rows
        for f, n in fc.items():
            tgt[base][f] += n * w / a.edges
        for kind, n in other[ph].items():
            tgt[base]["_" + kind] += n * w / a.edges
    order = ["top", "ck_addr", "ck_read", "ck_syn", "ck_min", "ck_merge", "ck_tab", "ck_pass2",
             "vn_setup", "vn_beta", "vn_sum", "vn_app", "vn_tv", "vn_vc", "vn_flags"]
    print(f"{name[:100]}")
    print(f"per pack-edge-iteration (static counts x waves / {a.edges} edges); cycles at "
          + ", ".join(f"{f} {COST[f]}" for f in FORMS))
    hdr = f"{'phase':10s} {'VALU':>7s} " + " ".join(f"{f:>6s}" for f in FORMS) + f" {'cyc':>7s} {'4cyc%':>6s} {'lds':>6s} {'salu':>6s}"
    print(hdr)
    tot = defaultdict(float)
    out = {}
    for base in order + sorted(set(rows) - set(order)):
        if base not in rows:
            continue
        r = rows[base]
        v = sum(r[f] for f in FORMS)
        cyc = sum(r[f] * COST[f] for f in FORMS)
        slow = sum(r[f] for f in FORMS if f != "v2")
        for f in FORMS + ["_lds", "_salu"]:
            tot[f] += r[f]
        out[base] = {f: round(r[f], 4) for f in FORMS + ["_lds", "_salu"]}
        print(f"{base:10s} {v:7.3f} " + " ".join(f"{r[f]:6.3f}" for f in FORMS)
              + f" {cyc:7.2f} {100 * slow / max(v, 1e-9):5.1f}% {r['_lds']:6.3f} {r['_salu']:6.3f}")
    v = sum(tot[f] for f in FORMS)
    cyc = sum(tot[f] * COST[f] for f in FORMS)
    print(f"{'total':10s} {v:7.3f} " + " ".join(f"{tot[f]:6.3f}" for f in FORMS)
          + f" {cyc:7.2f} {100 * sum(tot[f] for f in FORMS if f != 'v2') / v:5.1f}% {tot['_lds']:6.3f} {tot['_salu']:6.3f}")
    lv = sum(rows_last[b][f] for b in rows_last for f in FORMS)
    print(f"(the last iteration's variable phase instead: {lv:.3f} VALU per pack-edge)")
    if a.product:
        saved = {k: dict(v) for k, v in DUMP.items()}
        _, pc, _, _ = analyse(a.product, a.kernel)
        DUMP.clear()
        DUMP.update({k: defaultdict(int, v) for k, v in saved.items()})
        print("product build (unmarked), by the same propagation from the loop head (one phase):",
              {f: sum(c[f] for c in pc.values()) for f in FORMS})
    for phn in (a.dump.split(",") if a.dump else []):
        hist = sorted(DUMP[phn].items(), key=lambda kv: -kv[1])
        print(f"{phn}: " + ", ".join(f"{k} {v}" for k, v in hist))
    if a.json:
        json.dump({"kernel": name, "edges": a.edges, "dw": dw, "cwaves": a.cwaves,
                   "per_pack_edge_iter": out, "cost_cycles": COST}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
