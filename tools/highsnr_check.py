#!/usr/bin/env python3
"""Cross-check of the timed kernel against flood and the CPU oracle at high SNR on one config:
counters and per-frame flags of bsl/bsc and flood over B codewords, then the first failing frames
decoded by the oracle (APP at every iteration, last-iteration failure).

    python3 tools/highsnr_check.py C4 3.0,4.0 [--batch 1048576]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("snrs")
    ap.add_argument("--batch", type=int, default=1 << 20)
    a = ap.parse_args()
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from oracle import nms_oracle
    cfg = bench.CONFIGS[a.config]
    proto, g, W, cp = bench.load_problem(config=a.config)
    T, z = cfg["T"], cfg["z"]
    dev = torch.device("cuda", 0)
    dec = NMSDecoder(proto, z, W, 2, 5, device=dev, B_max=a.batch)
    dec.punct, dec.short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    for snr in [float(x) for x in a.snrs.split(",")]:
        llr = dec.awgn(a.batch, float(cp.sigma(snr)), seed=99)
        res = {}
        for k in ("fused", "flood"):
            r = dec.decode(llr, T=T, app=False, counters=True, flags=True, kernel=k)
            res[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy(), dec.last_kernel())
        same = np.array_equal(res["fused"][0], res["flood"][0]) and np.array_equal(res["fused"][1], res["flood"][1])
        fail = np.nonzero((res["fused"][1] >> 1) & 1)[0][:8]
        x = llr[torch.from_numpy(fail).to(dev)].cpu().numpy()
        o = nms_oracle.decode(x, proto, z, W.alpha, W.alpha_ucn, W.beta, T, 2, 5)
        small = dec.decode(torch.from_numpy(x).to(dev), T=T, app=True, flags=True)
        app_eq = np.array_equal(small.app.cpu().numpy(), o["app"])
        o_fail = o["hard"][T - 1].reshape(len(fail), -1).any(axis=1)
        wrong_bits = o["hard"][T - 1].reshape(len(fail), -1).sum(axis=1)
        print(f"{a.config} {snr} dB: {res['fused'][2]} counters {res['fused'][0].tolist()} flood "
              f"{res['flood'][0].tolist()} equal {same}; oracle APP equal on {len(fail)} failing "
              f"frames: {app_eq}, oracle fails them: {o_fail.tolist()}, wrong bits {wrong_bits.tolist()}",
              flush=True)
        if len(fail):
            hb = o["hard"][T - 1][0].reshape(-1)
            print("   first failing frame's wrong bit positions (1-based):", (np.nonzero(hb)[0] + 1).tolist()[:20],
                  flush=True)


if __name__ == "__main__":
    main()
