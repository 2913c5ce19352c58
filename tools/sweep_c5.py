#!/usr/bin/env python3
"""C5 error-floor sweep on one GPU (SURVEY §8 d C5: 5G NR BG1 n2112 R0.73, T=50, flat [3,0,3]
alpha=0.75 beta=1, puncture 1-144, shorten 1537-1584, QMS q5) through ``fer_sweep`` with
per-SNR checkpoints — the reference's FER loop (``Print_Functions.py:130-165``) at the
scale an error floor needs.

Stage 1 scans SNR coarsely (``--scan`` codewords per point); stage 2 decodes ``--deep``
codewords at every point whose scan FER is below ``--deep-below`` (and at the first point with
no error in the scan).  Each stage checkpoints to ``<out>/ckpt_<stage>.json`` every few batches
and resumes from it when rerun with the same arguments.  Writes ``<out>/sweep_c5.json``.

  python tools/sweep_c5.py --out gpurun_out/sweep_c5 [--scan 4194304] [--deep 1073741824]
  python tools/sweep_c5.py --out gpurun_out/c5_deep --deep-snrs 15.0 --deep 10737418240

``--config C2|C3|C4`` sweeps another SURVEY §8 d workload the same way (its trained weights and
channel ranges, bench.CONFIGS); the output is then ``<out>/sweep_<config>.json``.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/sweep_c5")
    ap.add_argument("--config", default="C5", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--snrs", default="2.5,3.0,3.25,3.5,3.75,4.0,4.25,4.5,5.0")
    ap.add_argument("--scan", type=int, default=1 << 22)
    ap.add_argument("--deep", type=int, default=1 << 30)
    ap.add_argument("--deep-below", type=float, default=1e-3)
    ap.add_argument("--batch", type=int, default=1 << 20)
    ap.add_argument("--deep-snrs", default="",
                    help="skip the scan: decode --deep codewords at each of these SNRs only")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.fer import fer_sweep

    os.makedirs(a.out, exist_ok=True)
    cfg = bench.CONFIGS[a.config]
    proto, g, W, cp = bench.load_problem(config=a.config)
    dev = torch.device("cuda", 0)
    dec = NMSDecoder(proto, cfg["z"], W, 2, 5, device=dev, B_max=a.batch)
    dec.punct, dec.short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    kernel = dec.kernel_info()[1]
    snrs = [float(x) for x in (a.deep_snrs or a.snrs).split(",")]
    sig = [float(x) for x in cp.sigma(np.asarray(snrs))]
    last = [time.time()]

    def progress(si, done, total):
        if time.time() - last[0] > 20:
            last[0] = time.time()
            print(f"  snr {snrs_cur[si]:.2f} dB: {done}/{total} codewords", flush=True)

    def point_seed(snr, stage):
        """1076 + 7919 x (SNR in millidecibels) + a per-stage offset: a function of the SNR value
        and the stage only (deep points do not reuse the scan's codewords either)."""
        return 1076 + 7919 * int(round(snr * 1000)) + (0 if stage == "scan" else 104729)

    def run(stage, idx, n):
        global snrs_cur
        snrs_cur = [snrs[i] for i in idx]
        t0 = time.time()
        # one Philox stream per SNR value (not per position in this call's list): the scan, the
        # deep stage and separate --deep-snrs runs of different SNRs never share noise
        res = fer_sweep(dec, [sig[i] for i in idx], n, a.batch, seed=1076, progress=progress,
                        checkpoint=os.path.join(a.out, f"ckpt_{stage}.json"), checkpoint_every=16,
                        resume=True, point_seeds=[point_seed(snrs[i], stage) for i in idx])
        dt = time.time() - t0
        rows = []
        for i, c in zip(idx, res):
            fe, fa = int(c.frame_err_last), int(c.frame_err_all)
            rows.append({"snr_db": snrs[i], "sigma": sig[i], "codewords": n,
                         "frame_err_last": fe, "fer_last": fe / n,
                         "frame_err_any_iter": fa, "fer": fa / n,
                         "bit_err_last": int(c.bit_err_last),
                         "ber_last": int(c.bit_err_last) / (n * dec.n_vars)})
            print(f"{stage} {snrs[i]:.2f} dB: FER_last {fe}/{n} = {fe / n:.3e}", flush=True)
        return rows, dt

    if a.deep_snrs:
        scan, t_scan, deep_idx = [], 0.0, list(range(len(snrs)))
    else:
        scan, t_scan = run("scan", list(range(len(snrs))), a.scan)
        deep_idx = [i for i, r in enumerate(scan) if 0 < r["fer_last"] < a.deep_below]
        zero = [i for i, r in enumerate(scan) if r["frame_err_last"] == 0]
        if zero:
            deep_idx.append(zero[0])
    deep, t_deep = run("deep", sorted(set(deep_idx)), a.deep) if deep_idx else ([], 0.0)
    n_total = a.scan * len(scan) + a.deep * len(set(deep_idx))
    if a.config == "C5":
        wl = ("C5: 5G_LDPC_R0.73_n_dec2304_n2112_k1536_z72_s1537_1584, QMS q5, T=50, "
              "flat [3,0,3] alpha=0.75 beta=1, puncture 1-144, shorten 1537-1584")
    else:
        sh = ",".join(str(x) for x in cfg["sharing"])
        wl = (f"{a.config}: {cfg['graph']}, QMS q5, T={cfg['T']}, sharing [{sh}] trained weights "
              f"({os.path.basename(cfg['weights'])})"
              + (f", puncture {cfg['punct'][0]}-{cfg['punct'][1]}" if "punct" in cfg else "")
              + (f", shorten {cfg['short'][0]}-{cfg['short'][1]}" if "short" in cfg else ""))
    out = {"workload": wl + ", on-GPU Philox AWGN (seed 1076 + 7919 x SNR in mdB, + 104729 in the "
                            "deep stage), all-zero codeword",
           "kernel": kernel, "scan": scan, "deep": deep,
           "seconds": {"scan": round(t_scan, 1), "deep": round(t_deep, 1)},
           "codewords_total": n_total,
           "codewords_per_s": round(n_total / max(t_scan + t_deep, 1e-9), 1),
           "note": "FER counters from fer_sweep (device int64 counters, calc_ber_fer "
                   "semantics: fer_last = frames wrong at the last iteration, fer = frames "
                   "wrong at every iteration); e2e includes the channel kernel"}
    with open(os.path.join(a.out, f"sweep_{a.config.lower()}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("kernel", "codewords_total", "codewords_per_s")}))


snrs_cur = []

if __name__ == "__main__":
    main()
