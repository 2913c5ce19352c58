#!/usr/bin/env python3
"""Throughput benchmark: decoded codewords/s, wman N576 R3/4, 20 NMS iterations.

One "step" = one decode of a resident batch (default B = 2^20 codewords per GPU, the
BASELINE.json configs[1] workload) with FER/BER counters accumulated on the device.  The
AWGN LLRs (3.5 dB, QMS q=5) are generated on the GPU before the timed region.
``python bench.py --gpus N --steps K --warmup W``: one rank per GPU, weak scaling (every rank
decodes its own B codewords, a disjoint slice of the global Philox stream).  Under
torch.distributed.run (WORLD_SIZE set) each process is one rank; run directly with N > 1, this
script starts the N ranks itself as fresh child processes (it never touches the GPU before
that) and exits with the first failing rank's status.

``--config C3|C4|C5`` runs the SURVEY §8 d companion workloads instead (802.11n, 5G BG2,
5G BG1); the default C2 line is the one the driver records.

Prints ONE JSON line (rank 0).  Besides the driver's fields it carries:
  roofline      the dominant kernel against the resource that binds it.  flood (state in HBM):
                bound "hbm", achieved = SURVEY §8 d bytes/codeword x B / kernel time (HIP
                events on the decode stream).  fused (state in LDS/VGPRs, VALU-issue bound):
                bound "valu", achieved = SQ_INSTS_VALU per launch (PMC of this build,
                profiles/traffic_<kernel>.json) / kernel time against one wave64 VALU issue
                per 2 cycles per SIMD; hbm_frac = measured PMC traffic / time / 8 TB/s and
                x_two_kernel_roofline = the §8 d figure / 8 TB/s (a speed-up over the
                two-kernel design at the HBM roofline) ride along.  traffic = PMC HBM
                bytes per launch (null without a profile of this kernel at this batch).
  cpu_baseline  the dense TF-graph-equivalent numpy restatement of the reference decoder
                (oracle/nms_dense.py) on the C1 sample (B=120, T=20, 3.5 dB), rank 0, N=1,
                sharded over one single-threaded worker process per core of the box's CPU
                share
  e2e_with_rng  K steps that each draw a fresh AWGN batch inside the timed region
                (ldpc_decode_awgn: generated in the decoder's prologue; SURVEY §8 d
                "separately time end-to-end with GPU RNG and counters")
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD (32 lanes
# per cycle, MI355X_MICROARCH.md "Wave scheduling") at 2.4 GHz, in wave-instructions per second
VALU_PEAK_WINST = 256 * 4 * 2.4e9 / 2
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")

# SURVEY.md §8 d workloads.  C2 is BASELINE.json's configs[1] (the driver's line).
CONFIGS = {
    "C2": dict(label="wman N576 R3/4", graph="wman_N0576_R34_z24", z=24, T=20, sharing=(3, 0, 3),
               weights="Weights/C0_wman_N0576_R34_z24_Opt_Weight_End20.txt", snr=3.5),
    "C3": dict(label="802.11n N648 R5/6", graph="802_11n_N648_R56_z27", z=27, T=50,
               sharing=(3, 3, 3), weights="Results/WIFI/Weights_Iter50.txt", snr=3.5),
    "C4": dict(label="5G BG2 n1024 R1/2", graph="5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640",
               z=64, T=20, sharing=(2, 2, 2),
               weights="Results/5G/5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640_Weight_End50.txt",
               snr=2.0, punct=(1, 128), short=(513, 640)),
    "C5": dict(label="5G BG1 n2112 R0.73", graph="5G_LDPC_R0.73_n_dec2304_n2112_k1536_z72_s1537_1584",
               z=72, T=50, sharing=(3, 0, 3), flat=(0.75, 1.0), snr=3.0, punct=(1, 144),
               short=(1537, 1584)),
}
GRAPH = CONFIGS["C2"]["graph"]
WEIGHTS = os.path.basename(CONFIGS["C2"]["weights"])


def survey_bytes_per_cw(E, N, z, T, ucn=False):
    """SURVEY.md §8 d: T * (3*E*z*4 + 4*N*z*4 + N*z/8 [+ N*z/8 with UCN])."""
    return T * (3 * E * z * 4 + 4 * N * z * 4 + N * z // 8 + (N * z // 8 if ucn else 0))


def load_problem(T=None, config="C2"):
    """(proto, TannerGraph, DecoderWeights, CodeParams) of a SURVEY §8 d workload."""
    from ldpc_error_floor_amd.code import CodeParams, TannerGraph, load_base_graph
    from ldpc_error_floor_amd.weights import expand_weights, flat_weights, read_weight_file
    c = CONFIGS[config]
    T = c["T"] if T is None else T
    z = c["z"]
    proto = load_base_graph(os.path.join(DATA, "BaseGraph", c["graph"] + ".txt"))
    g = TannerGraph(proto, z)
    if "weights" in c:
        wf = read_weight_file(os.path.join(DATA, c["weights"]))
        blocks = {k: v for k, v in wf.blocks.items() if c["sharing"][k] > 0}
        W = expand_weights(c["sharing"], blocks, T, g)
    else:                         # no trained weights ship for this code: flat [3,0,3]
        W = flat_weights(g, T, alpha=c["flat"][0], beta=c["flat"][1])
    ps, pe = c.get("punct", (0, 0))
    ss, se = c.get("short", (0, 0))
    return proto, g, W, CodeParams(proto, z, ps, pe, ss, se)


def _cpu_worker(proto, W, X, T, barrier, q):
    """One CPU-baseline process: builds the dense graph, waits for the others, decodes its
    slice of the C1 batch single-threaded (threadpoolctl), reports its decode time."""
    from threadpoolctl import threadpool_limits
    from oracle import nms_dense
    dg = nms_dense.DenseGraph(proto, 24)
    with threadpool_limits(limits=1):
        barrier.wait()
        t0 = time.perf_counter()
        if X.shape[0]:
            nms_dense.decode(X, proto, 24, W.alpha, W.alpha_ucn, W.beta, T, 2, 5, graph=dg)
        q.put(time.perf_counter() - t0)


def cpu_baseline(proto, g, W, cp, B=480, T=20, snr=3.5):
    """Dense TF-graph-equivalent numpy decoder on the C1 sample, sharded over worker processes.

    B = 480: four C1 batches (the first 480 codewords of the C1 stream), about 15 s of CPU work
    on the GPU box's 16 cores.  The batch is split into contiguous slices (fer.shard_range), one per worker process
    (spawned: fresh interpreters, nothing inherited from this process's HIP state), each
    decoding single-threaded after all have built their dense graph; value = B / the slowest
    worker's decode time.  Workers = the host cores this process may use, capped by the box's
    CPU share (OMP_NUM_THREADS, 16 on the GPU box): so `cores` is what actually ran."""
    import multiprocessing as mp
    from threadpoolctl import threadpool_limits
    from ldpc_error_floor_amd.channel import create_mix_epoch
    from ldpc_error_floor_amd.fer import shard_range
    from oracle import nms_oracle
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cores = len(os.sched_getaffinity(0))
    workers = max(1, min(cores, share if share > 0 else cores, B))
    sigma = float(cp.sigma(snr))
    wr, nr = np.random.RandomState(2044), np.random.RandomState(1076)
    X, _ = create_mix_epoch([sigma], wr, nr, B, g.N, g.N - g.M, 24, [], True, 2, 0, 0, 0, 0, 5, 20.0)
    X = X.reshape(B, -1).astype(np.float32)
    ctx = mp.get_context("spawn")
    barrier, q = ctx.Barrier(workers), ctx.Queue()
    procs = []
    for r in range(workers):
        b0, b1 = shard_range(B, r, workers)
        procs.append(ctx.Process(target=_cpu_worker, args=(proto, W, X[b0:b1], T, barrier, q)))
    for pr in procs:
        pr.start()
    times = [q.get(timeout=900) for _ in procs]
    for pr in procs:
        pr.join(timeout=60)
    dt = max(times)
    with threadpool_limits(limits=1):
        sg = nms_oracle.lifted_edges(proto, 24)
        t1 = time.perf_counter()
        nms_oracle.decode(X, proto, 24, W.alpha, W.alpha_ucn, W.beta, T, 2, 5, graph=sg)
        dt_sparse = time.perf_counter() - t1
    cpu = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), cpu)
    except OSError:
        pass
    return {"value": round(B / dt, 3), "unit": "codewords/s", "cores": workers, "kind": "port",
            "threads": f"{workers} worker processes x 1 thread (threadpoolctl), one contiguous "
                       f"slice of the batch each; {cores} cores in this process's affinity",
            "sample": f"C1 x {B // 120}: wman QMS q5 T={T}, the first {B} host-channel codewords at "
                      f"{snr} dB (seeds 2044/1076, compute_results order), dense TF-graph-equivalent "
                      f"numpy (oracle/nms_dense.py), slowest worker {dt:.2f} s (per worker: "
                      f"{min(times):.2f}-{dt:.2f} s, {sum(times):.1f} s of CPU in all)",
            "cpu_model": cpu,
            "sparse_oracle_cw_s_1thread": round(B / dt_sparse, 1)}


def launch_ranks(n):
    """Ranks 0..n-1 of this command as fresh child processes (ldpc_error_floor_amd.launch)."""
    from ldpc_error_floor_amd.launch import launch_ranks as _launch
    return _launch(__file__, sys.argv[1:], n, tag="bench.py")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="codewords per GPU per step")
    ap.add_argument("--kernel", default="auto", choices=["auto", "flood", "fused"])
    ap.add_argument("--snr", type=float, default=None, help="default: the config's SNR")
    ap.add_argument("--iters", type=int, default=None, help="default: the config's T")
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--decoding-type", type=int, default=2, choices=[0, 1, 2, 3],
                    help="0 sum-product, 1 MS fp32, 2 QMS (default), 3 MS without the zero nudge")
    ap.add_argument("--q-bit", type=int, default=5, choices=[6, 5, -5, 4, 3])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--all-kernels", action="store_true",
                    help="also time the non-default kernel and report it under 'kernels'")
    ap.add_argument("--no-companions", action="store_true",
                    help="skip the SURVEY 8d companion workloads (C3, C4, C5) a default one-GPU run "
                         "times after the headline and reports under 'companions'")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"bench.py: WORLD_SIZE={world} overrides --gpus {args.gpus}", file=sys.stderr)
    # one rank per GPU over RCCL; LDPC_BENCH_BACKEND=gloo rehearses the multi-rank code path
    # with several ranks on the same GPU (collectives then go through host copies)
    backend = os.environ.get("LDPC_BENCH_BACKEND", "nccl")
    ndev = torch.cuda.device_count()
    gpu = local if backend == "nccl" else local % max(ndev, 1)
    if backend == "nccl" and world > 1 and gpu >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {ndev} GPUs visible")
    dev = torch.device("cuda", gpu)
    torch.cuda.set_device(dev)
    # launched as a rank (torch.distributed.run, or this script's own launcher; WORLD_SIZE set,
    # 1 included): the process group is initialised and every collective below runs through it,
    # so a one-GPU run with WORLD_SIZE=1 exercises the same RCCL calls as the 8-GPU job
    dist_on = "WORLD_SIZE" in os.environ
    if dist_on:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        from ldpc_error_floor_amd.launch import fail_hook
        fail_hook(rank, "bench.py")

    def allreduce(t, op):
        """In-place all-reduce of a device tensor (host round trip for gloo)."""
        if not dist_on:
            return t
        if backend == "nccl":
            dist.all_reduce(t, op=op)
            return t
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
        return t

    def barrier():
        if dist_on:
            if backend == "nccl":
                dist.barrier(device_ids=[gpu])
            else:
                dist.barrier()

    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = CONFIGS[args.config]
    T = cfg["T"] if args.iters is None else args.iters
    snr = cfg["snr"] if args.snr is None else args.snr
    z = cfg["z"]
    punct, short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    proto, g, W, cp = load_problem(T, args.config)
    sigma = float(cp.sigma(snr))
    B = args.batch

    def run(kernel, e2e=False):
        dec = NMSDecoder(proto, z, W, args.decoding_type, args.q_bit, device=dev, kernel=kernel,
                         B_max=B)
        llr = dec.awgn(B, sigma, seed=1076, offset=rank * B, punct=punct, short=short)  # in HBM
        counters = torch.zeros(4, dtype=torch.int64, device=dev)
        name = dec.kernel_info(T)[1]
        stream = torch.cuda.current_stream(dev)
        for _ in range(args.warmup):      # (the warmups run the timed step: the e2e run's first
            if e2e:                       # decode_awgn builds and uploads the sampler tables)
                dec.decode_awgn(B, sigma, seed=1076, offset=rank * B, punct=punct, short=short,
                                T=T, counters=counters)
            else:
                dec.decode(llr, T=T, app=False, counters=counters)
        torch.cuda.synchronize(dev)
        counters.zero_()
        barrier()
        torch.cuda.synchronize(dev)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev1 = torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(args.steps):
            if e2e:                 # a fresh AWGN batch per step, generated by the decoder
                dec.decode_awgn(B, sigma, seed=1076 + i + 1, offset=rank * B, punct=punct,
                                short=short, T=T, counters=counters)
            else:
                dec.decode(llr, T=T, app=False, counters=counters)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        barrier()
        elapsed = allreduce(torch.tensor([t1 - t0], dtype=torch.float64, device=dev),
                            dist.ReduceOp.MAX if dist_on else None)
        cnt = allreduce(counters.clone(), dist.ReduceOp.SUM if dist_on else None)
        kernel_ms = ev0.elapsed_time(ev1) / args.steps
        return dict(name=name, elapsed=float(elapsed.item()), kernel_ms=kernel_ms,
                    counters=cnt.cpu().tolist(), design_bytes=dec.kernel_info(T)[0])

    primary = run(args.kernel)
    e2e = run(args.kernel, e2e=True)
    extra = {}
    if args.all_kernels:
        for k in ("flood", "fused"):
            try:
                r = run(k)
            except RuntimeError as e:
                extra[k] = {"error": str(e)}
                continue
            if r["name"] != primary["name"]:
                extra[r["name"]] = {"codewords_per_s": round(world * B * args.steps / r["elapsed"], 1),
                                    "ms_per_step": round(1e3 * r["elapsed"] / args.steps, 3)}

    t = primary["elapsed"]
    value = world * B * args.steps / t
    kernel_s = primary["kernel_ms"] / 1e3
    bytes_cw = survey_bytes_per_cw(g.E, g.N, z, T, ucn=cfg["sharing"][1] > 0)
    effective = bytes_cw * B / kernel_s / 1e9            # GB/s, SURVEY §8 d two-kernel bytes
    prof = load_profile(primary["name"], B)
    traffic = prof.get("hbm_bytes_per_launch") if prof else None
    fused = primary["name"] != "flood"
    if fused:
        vi = prof.get("valu_insts_per_launch") if prof else None
        rate = vi / kernel_s if vi else None
        vb = (prof.get("valu_busy") or {}) if prof else {}
        issue = round(rate / VALU_PEAK_WINST, 4) if rate else None
        roofline = {"bound": "valu",
                    "achieved": round(rate, 1) if rate else None, "peak": VALU_PEAK_WINST,
                    "unit": "wave-instructions/s",
                    "frac": issue,
                    "issue_frac": issue,
                    "traffic": traffic,
                    "hbm_frac": (round(traffic / kernel_s / 1e9 / HBM_PEAK_GBS, 4)
                                 if traffic else None),
                    "x_two_kernel_roofline": round(effective / HBM_PEAK_GBS, 2),
                    "valu_insts_per_launch": vi,
                    "valu_per_pack_edge_iter": (round(vi / ((B + 31) // 32 * g.E * z * T), 3)
                                                if vi and primary["name"].startswith(("bsl", "bsc"))
                                                else None),
                    "valu_busy": vb or None,
                    "lds_busy": prof.get("lds_busy") if prof else None,
                    "wait_any_frac": prof.get("wait_any_frac") if prof else None,
                    "profile": prof.get("source") if prof else None,
                    "profile_sources": prof.get("src_fingerprint") if prof else None}
        roofline["note"] = ("fused: all T iterations per codeword block in LDS/VGPRs; the only "
                            "HBM traffic is the LLR read, so the VALU pipe binds (the bit-sliced "
                            "bsl kernel: VALU issue and the LDS array together, lds_busy = "
                            "SQ_LDS_IDX_ACTIVE / (256 CUs x GRBM cycles / 8)). frac = "
                            "issue_frac = achieved / peak with achieved = SQ_INSTS_VALU per "
                            "launch (PMC of these sources: profile_sources = the sources' "
                            "fingerprint, else null) / this run's kernel time (HIP events) and "
                            "peak = one wave64 VALU issue per 2 cycles per SIMD at 2.4 GHz "
                            "(MI355X_MICROARCH.md), which only 2-cycle VOP1/VOP2 forms reach "
                            "(VOP3/SDWA/DPP and SGPR-operand forms take ~4.2 cycles, "
                            "DESIGN.md 3.3). valu_busy = the busy model of the same PMC run: "
                            "quad-cycles with a VALU issue (SQ_INSTS_VALU - "
                            "SQ_ACTIVE_INST_VALU2) / (1024 SIMDs x GRBM_GUI_ACTIVE/8/4), at the "
                            "clock of that run. x_two_kernel_roofline = this kernel's "
                            "codewords/s over the most a two-kernel HBM-resident decoder could "
                            "reach (SURVEY 8d bytes/codeword at 8 TB/s): a speed-up factor, not "
                            "a bandwidth fraction. valu_per_pack_edge_iter = VALU "
                            "wave-instructions / (32-codeword packs x lifted edges x T), the "
                            "bit-sliced kernels' instruction cost per edge update.")
    else:
        roofline = {"bound": "hbm", "achieved": round(effective, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(effective / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "note": "achieved = SURVEY 8d bytes/codeword x B / kernel time (HIP events)"}
    roofline.update({"kernel": primary["name"], "kernel_ms": round(primary["kernel_ms"], 3),
                     "algorithmic_bytes_per_cw": bytes_cw,
                     "design_bytes_per_cw": int(primary["design_bytes"])})
    c = primary["counters"]
    n_frames = world * B * args.steps
    wdesc = (f"trained weights ({os.path.basename(cfg['weights'])})" if "weights" in cfg
             else f"flat weights alpha={cfg['flat'][0]} beta={cfg['flat'][1]} (none ship)")
    pdesc = "".join([f", puncture {punct[0]}-{punct[1]}" if punct[0] else "",
                     f", shorten {short[0]}-{short[1]}" if short[0] else ""])
    sh = ",".join(str(x) for x in cfg["sharing"])
    mdesc = {0: "sum-product fp32", 1: "MS fp32", 3: "MS fp32 (no nudge)"}.get(args.decoding_type, f"QMS q{args.q_bit}")
    out = {
        "metric": f"decoded codewords/sec, {cfg['label']}, {T} NMS iters",
        "value": round(value, 1),
        "unit": "codewords/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * t / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "i32" if primary["name"].startswith(("bsl", "fused5")) else "f32",
        "data": f"synthetic (on-GPU Philox AWGN, all-zero codeword, {snr} dB, {mdesc} LLRs)",
        "config": {"workload": f"{args.config}: {cfg['graph']} {mdesc} T={T} sharing [{sh}] "
                               f"{wdesc}{pdesc}, B={B} codewords/GPU/step @ {snr} dB",
                   "batch_per_gpu": B, "iterations": T, "kernel": primary["name"],
                   "parallelism": f"dp{world}"},
        "roofline": roofline,
        "fer_at_snr": {"frames": n_frames, "fer_last": c[1] / n_frames,
                       "ber_last": c[0] / (n_frames * g.N * z)},
        "counters": {"bit_err_last": c[0], "frame_err_last": c[1], "frame_err_all": c[2],
                     "loss2": c[3], "seed": 1076, "rank_offsets": [r * B for r in range(world)]},
    }
    out["e2e_with_rng"] = {"codewords_per_s": round(world * B * args.steps / e2e["elapsed"], 1),
                           "ms_per_step": round(1e3 * e2e["elapsed"] / args.steps, 3)}
    if extra:
        out["kernels"] = extra
    if (world == 1 and rank == 0 and not args.no_cpu_baseline and args.config == "C2"
            and args.decoding_type == 2 and args.q_bit == 5):
        out["cpu_baseline"] = cpu_baseline(proto, g, W, cp, T=T)
    if (world == 1 and not dist_on and not args.no_companions and args.config == "C2"
            and args.decoding_type == 2 and args.q_bit == 5 and args.kernel == "auto"
            and args.iters is None and args.snr is None and args.batch == 1 << 20):
        # the other SURVEY 8d workloads (BASELINE configs[2..4]) timed in the same run, so the
        # driver's own bench line carries them: decode-only and with the channel generated in
        # the kernel, each at its own T, weights, SNR and B = 2^20 on this one GPU
        out["companions"] = {c: time_config(c, dev, steps=3, warmup=1) for c in ("C3", "C4", "C5")}
    if dist_on:
        out["process_group"] = {"backend": dist.get_backend(), "world": dist.get_world_size()}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


def time_config(config, dev, steps=3, warmup=1, B=1 << 20):
    """One GPU, one SURVEY 8d workload at its own T / weights / SNR: the decode of B resident
    codewords (HIP events on the decode stream) and the sweep step with the channel generated
    inside the decoder (ldpc_decode_awgn), with the counters of the timed decodes."""
    import torch
    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = CONFIGS[config]
    T, z, snr = cfg["T"], cfg["z"], cfg["snr"]
    punct, short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    proto, g, W, cp = load_problem(T, config)
    sigma = float(cp.sigma(snr))
    dec = NMSDecoder(proto, z, W, 2, 5, device=dev, B_max=B)
    llr = dec.awgn(B, sigma, seed=1076, punct=punct, short=short)
    counters = torch.zeros(4, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    res = {"workload": f"{config}: {cfg['graph']} QMS q5 T={T} @ {snr} dB, B={B}",
           "kernel": dec.kernel_info(T)[1]}
    for mode in ("decode", "e2e_with_rng"):
        for i in range(warmup):
            if mode == "decode":
                dec.decode(llr, T=T, app=False, counters=counters)
            else:
                dec.decode_awgn(B, sigma, seed=7 + i, punct=punct, short=short, T=T, counters=counters)
        torch.cuda.synchronize(dev)
        counters.zero_()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for i in range(steps):
            if mode == "decode":
                dec.decode(llr, T=T, app=False, counters=counters)
            else:
                dec.decode_awgn(B, sigma, seed=1077 + i, punct=punct, short=short, T=T, counters=counters)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        c = counters.cpu().tolist()
        r = {"codewords_per_s": round(B * steps / wall, 1), "ms_per_step": round(1e3 * wall / steps, 3),
             "kernel_ms": round(ev0.elapsed_time(ev1) / steps, 3),
             "frame_err_last": c[1], "fer_last": c[1] / (B * steps)}
        if mode == "decode":
            res.update(r)
        else:
            res[mode] = r
    del llr, dec
    torch.cuda.empty_cache()
    return res


def load_profile(name, batch):
    """profiles/traffic_<kernel>.json (tools/traffic_json.py) when it was taken at this batch
    of a build from the current native sources (its src_fingerprint); None otherwise, so no
    PMC figure of another build is reported beside this run's timing."""
    from ldpc_error_floor_amd.build import source_fingerprint
    safe = "".join(ch if (ch.isalnum() or ch in "_.-") else "_" for ch in name)
    path = os.path.join(ROOT, "profiles", f"traffic_{safe}.json")
    try:
        with open(path) as f:
            tj = json.load(f)
    except (OSError, ValueError):
        return None
    if int(tj.get("batch", -1)) != batch or tj.get("src_fingerprint") != source_fingerprint():
        return None
    return tj


if __name__ == "__main__":
    main()
