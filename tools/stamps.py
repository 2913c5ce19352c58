#!/usr/bin/env python3
"""Analyse a fused5 LDPC_DIAG_STAMPS dump (see report_stamps in ldpc_fused5.hip).

  LDPC_DIAG_STAMPS=gpurun_out/st.bin python bench.py --steps 1 --warmup 0 --no-cpu-baseline
  python3 tools/stamps.py gpurun_out/st.bin --nblocks 65536 --T 20 [--launch 0]

Marks are 100 MHz s_memrealtime ticks (10 ns).  Prints per-phase and per-iteration means, and
for each CU (XCC, SE, SH, CU from HW_ID) how its workgroups overlapped in time.
"""
import argparse

import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--nblocks", type=int, required=True)
    ap.add_argument("--T", type=int, default=20)
    ap.add_argument("--launch", type=int, default=0)
    a = ap.parse_args()
    raw = np.fromfile(a.path, dtype=np.uint64)
    per = a.nblocks * 32
    nl = raw.size // per
    print(f"{nl} launches in file")
    s = raw[a.launch * per:(a.launch + 1) * per].reshape(a.nblocks, 32).astype(np.int64)
    t0 = s[:, 0].min()
    us = lambda x: x / 100.0
    def ph(name, i, j):
        d = s[:, j] - s[:, i]
        print(f"{name:26s} mean {us(d.mean()):8.2f} us  p50 {us(np.median(d)):8.2f}  "
              f"p99 {us(np.percentile(d, 99)):8.2f}")
    ph("prologue", 0, 1)
    ph("edge setup", 1, 2)
    ph("it0 pass1 (wave0)", 2, 5)
    ph("it0 pass2+sync", 5, 6)
    ph("it0 VN+sync", 6, 9)
    T = a.T
    TS = min(T, 22)                      # the kernel stamps iteration starts t < 22 only
    its = [s[:, 9 + t] - s[:, 8 + t] for t in range(TS - 1)]
    if TS == T:
        its.append(s[:, 30] - s[:, 8 + T - 1])
    print("iteration means (us):", " ".join(f"{us(x.mean()):.2f}" for x in its))
    ph("whole", 0, 30)
    span = s[:, 30].max() - t0
    print(f"launch span {us(span):.1f} us")
    hw = s[:, 31]
    xcc = hw >> 32
    cu = (xcc << 8) | ((hw >> 8) & 0xFF)
    ucu = np.unique(cu)
    print(f"{ucu.size} distinct CUs, {np.unique(xcc).size} XCCs; blocks per CU "
          f"min {np.bincount(np.searchsorted(ucu, cu)).min()} max {np.bincount(np.searchsorted(ucu, cu)).max()}")
    # concurrency seen by each block at its start / per-iteration, on its CU
    conc = np.zeros(a.nblocks, dtype=np.int64)
    iters_by_conc = {}
    for c in ucu[:64]:
        idx = np.nonzero(cu == c)[0]
        st, en = s[idx, 0], s[idx, 30]
        for k, b in enumerate(idx):
            conc[b] = int(((st <= st[k]) & (en > st[k])).sum())
    sel = conc > 0
    for c in np.unique(conc[sel]):
        m = sel & (conc == c)
        print(f"blocks starting with {c} resident on their CU (incl. self): {m.sum():6d}, "
              f"it0 {us((s[m, 9] - s[m, 8]).mean()):.2f} us, it5 {us((s[m, 14] - s[m, 13]).mean()):.2f} us")
    # one CU's timeline
    c = ucu[0]
    idx = np.nonzero(cu == c)[0]
    idx = idx[np.argsort(s[idx, 0])][:8]
    print("first blocks on one CU (start, end, us from launch start; hw id):")
    for b in idx:
        print(f"  block {b:6d}  {us(s[b, 0] - t0):9.2f} -> {us(s[b, 30] - t0):9.2f}  "
              f"it starts " + " ".join(f"{us(s[b, 8 + t] - t0):.1f}" for t in range(0, min(T, 22), 4))
              + f"  hw {int(hw[b]) & 0xFFFFFFFF:08x}")


if __name__ == "__main__":
    main()
