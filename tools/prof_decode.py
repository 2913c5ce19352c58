#!/usr/bin/env python3
"""Run a few decodes of one kernel for rocprofv3 (kernel trace / PMC counters).
usage: python3 tools/prof_decode.py --kernel fused --batch 262144 --reps 3 [--config C5]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="fused")
    ap.add_argument("--batch", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--snr", type=float, default=None, help="default: the config's SNR")
    ap.add_argument("--config", default="C2", help="a bench.py SURVEY 8d workload (C2..C5)")
    ap.add_argument("--decoding-type", type=int, default=2)
    ap.add_argument("--q-bit", type=int, default=5)
    ap.add_argument("--e2e", action="store_true",
                    help="decode_awgn (the channel kernel + the decoder) instead of decode")
    a = ap.parse_args()
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = bench.CONFIGS[a.config]
    proto, g, W, cp = bench.load_problem(config=a.config)
    snr = cfg["snr"] if a.snr is None else a.snr
    dec = NMSDecoder(proto, cfg["z"], W, a.decoding_type, a.q_bit, kernel=a.kernel, B_max=a.batch)
    llr = dec.awgn(a.batch, float(cp.sigma(snr)), seed=1076, punct=cfg.get("punct", (0, 0)),
                   short=cfg.get("short", (0, 0)))
    cnt = torch.zeros(4, dtype=torch.int64, device=llr.device)
    for i in range(a.reps):
        if a.e2e:
            dec.decode_awgn(a.batch, float(cp.sigma(snr)), seed=1077 + i, punct=cfg.get("punct", (0, 0)),
                            short=cfg.get("short", (0, 0)), T=cfg["T"], counters=cnt)
        else:
            dec.decode(llr, T=cfg["T"], app=False, counters=cnt)
    torch.cuda.synchronize()
    print("counters", cnt.tolist(), "kernel", dec.kernel_info()[1])


if __name__ == "__main__":
    main()
