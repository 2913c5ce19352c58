#!/usr/bin/env python3
"""Error-floor FER sweep (BASELINE.json configs[4]: 5G NR BG1 n2112 R0.73, T=50, "error-floor
FER sweep to 1e-9 on 8x MI355X"; SURVEY §8 d C5: flat [3,0,3] alpha=0.75 beta=1, puncture
1-144, shorten 1537-1584, QMS q5) through ``fer_sweep`` with per-SNR checkpoints — the
reference's FER loop (``Print_Functions.py:130-165``) at the scale an error floor needs, one
process per GPU as the reference runs (``main_Base.py:14-15``).

Stage 1 scans SNR coarsely (``--scan`` codewords per point); stage 2 decodes ``--deep``
codewords at every point whose scan FER is below ``--deep-below`` (and at the first point with
no error in the scan).  Each stage checkpoints to ``<out>/ckpt_<stage>.json`` (rank r > 0:
``.rank<r>``) every few batches and resumes from it when rerun with the same arguments; a
resume at another world size is refused (the key holds the partition).  Rank 0 writes
``<out>/sweep_<config>.json``.

  python tools/sweep_c5.py --out gpurun_out/sweep_c5 [--scan 4194304] [--deep 1073741824]
  python tools/sweep_c5.py --gpus 8 --out gpurun_out/c5_deep --deep-snrs 15.0 --deep 85899345920

``--gpus N`` (N > 1, no WORLD_SIZE in the environment): starts ranks 0..N-1 of this command as
fresh child processes (``ldpc_error_floor_amd.launch``; never an exec); under
``torch.distributed.run`` each process is one rank.  Every rank joins an ``nccl`` (RCCL) group
on its LOCAL_RANK's GPU (``LDPC_SWEEP_BACKEND=gloo`` rehearses on CPU).  A point's codewords are
split contiguously over the ranks (``fer.shard_range``) and each codeword's noise is the Philox
stream at its *global* index, so any world size decodes the same codewords and returns the same
counters; the one collective per stage is ``fer_sweep``'s all_reduce of the [nSNR, 4] counter
block (plus a max of the stage time).

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


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/sweep_c5")
    ap.add_argument("--config", default="C5", choices=["C2", "C3", "C4", "C5"])
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU)")
    ap.add_argument("--snrs", default="2.5,3.0,3.25,3.5,3.75,4.0,4.25,4.5,5.0")
    ap.add_argument("--scan", type=int, default=1 << 22)
    ap.add_argument("--deep", type=int, default=1 << 30)
    ap.add_argument("--deep-below", type=float, default=1e-3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per rank per decode")
    ap.add_argument("--uncor", action="store_true",
                    help="collect the frames wrong at every iteration into <out>/Uncor_<stage>.txt "
                         "(the Uncor.txt format main_Post.py reads; one merged file at any --gpus)")
    ap.add_argument("--deep-snrs", default="",
                    help="skip the scan: decode --deep codewords at each of these SNRs only")
    a = ap.parse_args(argv)
    if a.gpus < 1:
        ap.error("--gpus must be >= 1")
    return a


def point_seed(snr, stage):
    """1076 + 7919 x (SNR in millidecibels) + a per-stage offset: a function of the SNR value
    and the stage only (deep points do not reuse the scan's codewords either)."""
    return 1076 + 7919 * int(round(snr * 1000)) + (0 if stage == "scan" else 104729)


def workload(config, cfg):
    if config == "C5":
        return ("C5: 5G_LDPC_R0.73_n_dec2304_n2112_k1536_z72_s1537_1584, QMS q5, T=50, "
                "flat [3,0,3] alpha=0.75 beta=1, puncture 1-144, shorten 1537-1584")
    sh = ",".join(str(x) for x in cfg["sharing"])
    return (f"{config}: {cfg['graph']}, QMS q5, T={cfg['T']}, sharing [{sh}] trained weights "
            f"({os.path.basename(cfg['weights'])})"
            + (f", puncture {cfg['punct'][0]}-{cfg['punct'][1]}" if "punct" in cfg else "")
            + (f", shorten {cfg['short'][0]}-{cfg['short'][1]}" if "short" in cfg else ""))


def main(argv=None, make_decoder=None):
    """``make_decoder(config, device, batch)``: the decoder to sweep with (default: the HIP
    ``NMSDecoder`` of the config; the CPU tests pass an oracle-backed stand-in)."""
    a = parse(argv)
    from ldpc_error_floor_amd.launch import init_rank_group, launch_ranks, rank_info
    launched, world, rank, local = rank_info()
    if a.gpus > 1 and not launched:
        return launch_ranks(__file__, sys.argv[1:] if argv is None else argv, a.gpus,
                            tag="sweep_c5.py")
    if launched and world != a.gpus and rank == 0:
        print(f"sweep_c5.py: WORLD_SIZE={world} overrides --gpus {a.gpus}", file=sys.stderr)
    import numpy as np
    import torch
    import torch.distributed as dist
    import bench
    from ldpc_error_floor_amd.fer import fer_sweep

    backend = os.environ.get("LDPC_SWEEP_BACKEND", "nccl")
    dev = init_rank_group(backend, local)
    if launched:
        from ldpc_error_floor_amd.launch import fail_hook
        fail_hook(rank, "sweep_c5.py")
    os.makedirs(a.out, exist_ok=True)
    cfg = bench.CONFIGS[a.config]
    proto, g, W, cp = bench.load_problem(config=a.config)
    if make_decoder is None:
        from ldpc_error_floor_amd.decoder import NMSDecoder
        dec = NMSDecoder(proto, cfg["z"], W, 2, 5, device=dev, B_max=a.batch)
    else:
        dec = make_decoder(a.config, dev, a.batch)
    dec.punct, dec.short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    kernel = dec.kernel_info()[1] if hasattr(dec, "kernel_info") else type(dec).__name__
    snrs = [float(x) for x in (a.deep_snrs or a.snrs).split(",")]
    sig = [float(x) for x in cp.sigma(np.asarray(snrs))]
    last = [time.time()]
    cur = []

    def progress(si, done, total):
        if rank == 0 and time.time() - last[0] > 20:
            last[0] = time.time()
            print(f"  snr {cur[si]:.2f} dB: rank 0 {done}/{total} codewords", flush=True)

    def stage_time(dt):
        """The slowest rank's time for the stage (the job's time)."""
        if not dist.is_initialized():
            return dt
        on_dev = dist.get_backend() == "nccl"
        t = torch.tensor([dt], dtype=torch.float64, device=dev if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def run(stage, idx, n):
        cur[:] = [snrs[i] for i in idx]
        t0 = time.time()
        # one Philox stream per SNR value (not per position in this call's list): the scan, the
        # deep stage and separate --deep-snrs runs of different SNRs never share noise
        res = fer_sweep(dec, [sig[i] for i in idx], n, a.batch, seed=1076, progress=progress,
                        checkpoint=os.path.join(a.out, f"ckpt_{stage}.json"), checkpoint_every=16,
                        resume=True, point_seeds=[point_seed(snrs[i], stage) for i in idx],
                        uncor_path=os.path.join(a.out, f"Uncor_{stage}.txt") if a.uncor else None)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)
        dt = stage_time(time.time() - t0)
        rows = []
        for i, c in zip(idx, res):
            fe, fa = int(c.frame_err_last), int(c.frame_err_all)
            rows.append({"snr_db": snrs[i], "sigma": sig[i], "codewords": n,
                         "frame_err_last": fe, "fer_last": fe / n,
                         "frame_err_any_iter": fa, "fer": fa / n,
                         "bit_err_last": int(c.bit_err_last),
                         "ber_last": int(c.bit_err_last) / (n * dec.n_vars)})
            if rank == 0:
                print(f"{stage} {snrs[i]:.2f} dB: FER_last {fe}/{n} = {fe / n:.3e}", flush=True)
        return rows, dt

    try:
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
        out = {"workload": workload(a.config, cfg) +
               ", on-GPU Philox AWGN (seed 1076 + 7919 x SNR in mdB, + 104729 in the deep stage, "
               "indexed by the global codeword number), all-zero codeword",
               "kernel": kernel, "n_gpus": world,
               "process_group": ({"backend": dist.get_backend(), "world": dist.get_world_size()}
                                 if dist.is_initialized() else None),
               "batch_per_rank": a.batch, "scan": scan, "deep": deep,
               "seconds": {"scan": round(t_scan, 1), "deep": round(t_deep, 1)},
               "codewords_total": n_total,
               "codewords_per_s": round(n_total / max(t_scan + t_deep, 1e-9), 1),
               "uncor_files": ([f"Uncor_{st}.txt" for st, rows in (("scan", scan), ("deep", deep)) if rows]
                               if a.uncor else None),
               "note": "FER counters from fer_sweep (device int64 counters summed over the ranks, "
                       "calc_ber_fer semantics: fer_last = frames wrong at the last iteration, "
                       "fer = frames wrong at every iteration); e2e includes the channel kernel; "
                       "seconds = the slowest rank's"}
        if rank == 0:
            with open(os.path.join(a.out, f"sweep_{a.config.lower()}.json"), "w") as f:
                json.dump(out, f, indent=1)
            print(json.dumps({k: out[k] for k in ("kernel", "n_gpus", "codewords_total",
                                                  "codewords_per_s")}), flush=True)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
