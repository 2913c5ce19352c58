"""LDS bank model of the bit-sliced (bsl) variable phase, for layout experiments (CPU only).

Restates ldpc_bs.hip's slot layout (slot_layout) and variable-lane order (degree-sorted chunks of
64) and counts, per half-wave (32 lanes) and edge round f, the LDS cycles of one slot-word access:
the most distinct dword addresses on one bank (bank = dword mod 32).  Compares the graph's edge
order, the per-lane edge reorder (host::order_variable_edges) and a search that also swaps
equal-degree variables between half-waves.

  python tools/bank_model.py [wman_N0576_R34_z24 24 4]
"""
import os
import random
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from ldpc_error_floor_amd.code import TannerGraph, load_base_graph  # noqa: E402


def slot_layout(g, LPC):
    sep = 32 // LPC

    def ok(A):
        for d in range(1, LPC):
            r = (d * A) % 32
            if min(r, 32 - r) < sep:
                return False
        return True
    lay, cur = [], 0
    for i in range(g.M):
        deg = int(g.cn_deg[i])
        first = cur
        if i > 0:
            first += ((lay[-1][0] + g.z - cur) % 32 + 32) % 32
        A = ((deg + LPC - 1) // LPC) * g.z
        while not ok(A):
            A += 1
        last_rows = max((deg - (LPC - 1) + LPC - 1) // LPC, 0)
        cur = first + (LPC - 1) * A + last_rows * g.z
        lay.append((first, A))
    return lay


def lane_slots(g, lay, LPC):
    z = g.z
    out = []
    for v in range(g.N * z):
        j, hh = divmod(v, z)
        s = []
        for pe in np.nonzero(g.pe_col == j)[0]:
            i = int(g.pe_row[pe])
            kk = int(pe - g.row_ptr[i])
            hc = (hh - int(g.pe_shift[pe])) % z
            s.append(lay[i][0] + (kk % LPC) * lay[i][1] + (kk // LPC) * z + hc)
        out.append(s)
    return out


def round_cost(lanes, f):
    cnt = {}
    seen = set()
    for s in lanes:
        a = s[f] if f < len(s) else -1          # -1: the shared zero slot (broadcast)
        if a in seen:
            continue
        seen.add(a)
        b = a % 32 if a >= 0 else 31
        cnt[b] = cnt.get(b, 0) + 1
    # cycles, with the sum of squared bank loads as the tie-break (as order_variable_edges)
    return max(cnt.values()) * 4096 + sum(c * c for c in cnt.values())


def total(halves, rounds):
    return sum(round_cost(h, f) // 4096 for h, r in zip(halves, rounds) for f in range(r))


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "wman_N0576_R34_z24"
    z = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    LPC = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    g = TannerGraph(load_base_graph(os.path.join(os.path.dirname(__file__), "..", "ldpc_error_floor_amd", "data", "BaseGraph", name + ".txt")), z)
    lay = slot_layout(g, LPC)
    slots = lane_slots(g, lay, LPC)
    nv = len(slots)
    order = sorted(range(nv), key=lambda v: -len(slots[v]))
    lanes = [list(slots[v]) for v in order]
    halves = [lanes[h:h + 32] for h in range(0, nv, 32)]
    rounds = [max(len(slots[order[64 * (h // 2)]]), 0) for h in range(len(halves))]
    print("graph order:", total(halves, rounds), " lower bound:", sum(rounds))
    rng = random.Random(1)
    # edge reorder only
    for h, r in zip(halves, rounds):
        for _ in range(4000):
            l = rng.randrange(len(h))
            if len(h[l]) < 2:
                continue
            f1, f2 = rng.sample(range(len(h[l])), 2)
            c0 = round_cost(h, f1) + round_cost(h, f2)
            h[l][f1], h[l][f2] = h[l][f2], h[l][f1]
            if round_cost(h, f1) + round_cost(h, f2) > c0:
                h[l][f1], h[l][f2] = h[l][f2], h[l][f1]
    print("edge reorder:", total(halves, rounds))
    # plus swaps of equal-degree variables between half-waves
    byd = {}
    for hi, h in enumerate(halves):
        for l, s in enumerate(h):
            byd.setdefault(len(s), []).append((hi, l))
    for _ in range(int(os.environ.get('ITERS', 200000))):
        if rng.random() < 0.5:
            d = rng.choice(list(byd))
            if len(byd[d]) < 2:
                continue
            (h1, l1), (h2, l2) = rng.sample(byd[d], 2)
            if h1 == h2:
                continue
            c0 = sum(round_cost(halves[h1], f) for f in range(rounds[h1])) + \
                sum(round_cost(halves[h2], f) for f in range(rounds[h2]))
            halves[h1][l1], halves[h2][l2] = halves[h2][l2], halves[h1][l1]
            c1 = sum(round_cost(halves[h1], f) for f in range(rounds[h1])) + \
                sum(round_cost(halves[h2], f) for f in range(rounds[h2]))
            if c1 > c0:
                halves[h1][l1], halves[h2][l2] = halves[h2][l2], halves[h1][l1]
        else:
            hi = rng.randrange(len(halves))
            h = halves[hi]
            l = rng.randrange(len(h))
            if len(h[l]) < 2:
                continue
            f1, f2 = rng.sample(range(len(h[l])), 2)
            c0 = round_cost(h, f1) + round_cost(h, f2)
            h[l][f1], h[l][f2] = h[l][f2], h[l][f1]
            if round_cost(h, f1) + round_cost(h, f2) > c0:
                h[l][f1], h[l][f2] = h[l][f2], h[l][f1]
    print("edge reorder + variable swaps:", total(halves, rounds))


if __name__ == "__main__":
    main()
