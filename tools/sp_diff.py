#!/usr/bin/env python3
"""Diagnostic: sum-product (decoding_type 0) GPU flood decode vs the SP golden fixtures."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_case  # noqa: E402

from ldpc_error_floor_amd.decoder import NMSDecoder  # noqa: E402

for name in ("wman_303_sp_snr2.5", "wman_333_sp_snr2.0", "g5bg2_222_sp_snr2.0"):
    c = load_case(name)
    Nt = c["Nt"] if c["Nt"] < c["g"].N else 0
    dec = NMSDecoder(c["g"].proto, c["z"], c["W"], 0, 5, target_node=Nt, kernel="flood")
    app = dec.decode(c["llr"], app=True).app.cpu().numpy()
    ref = c["app"]
    d = np.abs(app - ref)
    for t in (0, 1, c["T"] // 2, c["T"] - 1):
        dt = d[t]
        print(f"{name} t={t}: max {dt.max():.3g} p99.9 {np.percentile(dt, 99.9):.3g} "
              f"p99 {np.percentile(dt, 99):.3g} mean {dt.mean():.3g}")
    flips = (app >= 0) != (ref >= 0)
    for m in (0.0, 0.1, 0.5, 1.0):
        print(f"   hard flips where |ref| >= {m}: {int(flips[np.abs(ref) >= m].sum())} / {flips.size}")
    print("   frames wrong@last ref", int((ref[-1] >= 0).any(axis=1).sum()), "gpu",
          int((app[-1] >= 0).any(axis=1).sum()))
