#!/usr/bin/env python3
"""End-to-end step time with the on-GPU channel in line (ldpc_decode_awgn: channel kernel, then
the bit-sliced decode) against the channel of batch i + 1 generated on a second stream while
batch i decodes (two LLR buffers), on the sweep's codeword stream (one seed, offsets += B).

    python3 tools/overlap_probe.py [C2 C5 ...] [--steps K] [--batch B]

Measured (profiles/r3/overlap/overlap.log): no gain, so fer_sweep keeps overlap=False."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["C2", "C5"])
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1 << 20)
    args = ap.parse_args()
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.fer import pipelined_channel_decode
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for cfg in args.configs:
        c = bench.CONFIGS[cfg]
        proto, g, W, cp = bench.load_problem(None, cfg)
        B, K = args.batch, args.steps
        dec = NMSDecoder(proto, c["z"], W, 2, 5, device=dev, B_max=B)
        dec.punct, dec.short = c.get("punct", (0, 0)), c.get("short", (0, 0))
        sigma = float(cp.sigma(c["snr"]))
        jobs = [(0, i * B, B) for i in range(K)]

        def seq(cnt):
            for _, pos, b in jobs:
                dec.decode_awgn(b, sigma, 1076, offset=pos, counters=cnt)

        def pipe(cnt):
            pipelined_channel_decode(dec, jobs, lambda si: (sigma, 1076), cnt=lambda si: cnt)

        res = {}
        for name, fn in (("inline", seq), ("overlap", pipe), ("inline", seq), ("overlap", pipe)):
            cnt = torch.zeros(4, dtype=torch.int64, device=dev)
            fn(cnt)                                  # warm-up (tables, buffers)
            torch.cuda.synchronize()
            cnt.zero_()
            t0 = time.perf_counter()
            fn(cnt)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / K
            res.setdefault(name, []).append(dt)
            print(f"{cfg} {name}: {1e3 * dt:.3f} ms/step, {B / dt / 1e6:.1f} M cw/s, "
                  f"counters {cnt.cpu().tolist()}", flush=True)
        print(f"{cfg} kernel {dec.kernel_info()[1]}: inline {1e3 * min(res['inline']):.3f} ms, "
              f"overlap {1e3 * min(res['overlap']):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
