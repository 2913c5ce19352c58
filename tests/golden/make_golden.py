#!/usr/bin/env python3
"""Generate the golden fixtures in ``tests/golden/*.npz`` from the reference's own code.

Runs ONLY in the build container (needs ``/root/reference``; override with
``LDPC_REFERENCE``).  Nothing from the reference is copied into the repo: this script
imports it, runs it, and saves inputs + outputs as data.

* ``Print_Functions`` (channel ``create_mix_epoch``, ``calc_ber_fer``, ``compute_results``)
  is imported and run unmodified (it needs only numpy).
* ``Main_Functions`` (``init_parameter``, ``init_connecting_matrix``, ``weight_init``,
  ``build_neural_network``) imports ``tensorflow.compat.v1``, which is not installed; it
  runs unmodified on top of ``_tf_standin`` (eager numpy equivalents of the TF ops used;
  exact in QMS mode, see that module's docstring).

Usage:  python tests/golden/make_golden.py [--only NAME ...]
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("LDPC_REFERENCE", "/root/reference")
F32 = np.float32


def import_reference():
    sys.path.insert(0, HERE)
    import _tf_standin
    _tf_standin.install()
    sys.path.insert(0, REF)
    import Main_Functions as MF      # noqa: E402
    import Print_Functions as PF     # noqa: E402
    return MF, PF


def load_proto(name):
    return np.loadtxt(os.path.join(REF, "BaseGraph", name + ".txt"), int, delimiter="\t")


def lifted_H(proto, z):
    """Dense lifted parity-check matrix, written independently of the package code."""
    M, N = proto.shape
    H = np.zeros((M * z, N * z), np.uint8)
    for i in range(M):
        for j in range(N):
            if proto[i, j] != -1:
                s = proto[i, j] % z
                for h in range(z):
                    H[i * z + h, j * z + (h + s) % z] = 1
    return H


def read_blocks(path):
    """Raw per-kind rows of a weight file (header-directed; float64)."""
    lines = open(path).read().split("\n")
    sharing = [int(x) for x in lines[0].split()]
    blocks, pos = {}, 1
    for kind, s in enumerate(sharing):
        if s <= 0:
            continue
        while not lines[pos].strip():
            pos += 1
        rows = []
        while pos < len(lines) and lines[pos].strip():
            rows.append([float(x) for x in lines[pos].split()])
            pos += 1
        blocks[kind] = np.array(rows)
    return sharing, blocks


class Graph:
    def __init__(self, MF, proto, z, sigma_snr=(3.0,), ps=0, pe=0, ss=0, se=0):
        self.MF = MF
        self.proto = proto
        self.z = z
        (self.M, self.N, self.base, self.cn_deg, self.vn_deg, self.E, self.rate,
         self.sigma) = MF.init_parameter(proto, np.asarray(sigma_snr, float), z, ps, pe, ss, se)
        t0 = time.time()
        self.mats = MF.init_connecting_matrix(proto, self.base, self.N, self.M, self.E, z,
                                              self.vn_deg, self.cn_deg, ps, pe)
        print(f"  init_connecting_matrix {proto.shape} z={z}: {time.time() - t0:.1f}s", flush=True)


def run_graph(g, X, Y, sharing, decoding_type, q_bit, T, var_rows, target_node,
              fixed_iter=0, training_iter_start=0, sampling_type=0, loss_type=2, etha=0.0):
    """Execute the reference graph eagerly; returns net_dict (concrete arrays)."""
    B = X.shape[0]
    net = {"xa": np.asarray(X, F32).reshape(B, g.N, g.z), "ya": np.asarray(Y, F32),
           "etha": etha, "learn_rate": 0.0,
           "LLRa0": np.zeros((B, g.z, g.E), F32)}
    for kind, rows in var_rows.items():
        for t in range(rows.shape[0]):
            net[f"var_{kind}_{t}"] = np.asarray(rows[t], F32)
    for t in range(T):
        net = g.MF.build_neural_network(net, list(sharing), decoding_type, sampling_type,
                                        loss_type, target_node, t, T, fixed_iter, 0,
                                        training_iter_start, T, g.N, g.M, g.E, g.z, B,
                                        *g.mats, q_bit, 20.0)
    return net


def var_rows_from_blocks(sharing, blocks, T, fixed_iter, M, N, E):
    """var_{i}_{t} arrays for t < n_iter from header-directed blocks (first rows)."""
    out = {}
    for kind, s in enumerate(sharing):
        if s <= 0:
            continue
        n_iter = T if s in (1, 2, 3) else fixed_iter + 1
        width = {1: E, 4: E, 3: 1}.get(s, M if kind < 2 else N)
        rows = blocks[kind][:n_iter].astype(F32)
        assert rows.shape == (n_iter, width), (kind, rows.shape, n_iter, width)
        out[kind] = rows
    return out


def save_case(name, g, X, net, T, B, target_node, meta, var_rows, decoding_type):
    Nt = target_node if target_node > 0 else g.N
    app = np.asarray(net["ya_output_all"], F32).reshape(T, B, Nt * g.z)
    full = np.stack([np.asarray(net[f"ya_output{t}"], F32).reshape(B, g.N * g.z)
                     for t in range(T)])
    assert np.array_equal(full[:, :, :Nt * g.z], app)
    hard = (full >= 0).astype(np.uint8)
    H = lifted_H(g.proto, g.z)
    synd = (np.einsum("tbv,cv->tbc", hard.astype(np.int64), H.astype(np.int64)) & 1).astype(np.uint8)
    d = dict(meta)
    d["proto"] = g.proto.astype(np.int32)
    d["llr"] = np.asarray(X, F32).reshape(B, g.N * g.z)
    if decoding_type == 2:
        a2 = app * 2
        assert np.array_equal(a2, np.round(a2)) and np.abs(a2).max() <= 127
        d["app_x2"] = a2.astype(np.int8)
    else:
        d["app"] = app
    d["hard_packed"] = np.packbits(hard, axis=-1)
    d["synd_packed"] = np.packbits(synd, axis=-1)
    d["n_vars"] = g.N * g.z
    d["n_checks"] = g.M * g.z
    d["loss"] = np.float32(net["lossa"]) if "lossa" in net else np.float32(np.nan)
    for kind, rows in var_rows.items():
        d[f"w{kind}"] = rows
    d["rate"] = np.float64(g.rate)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **d)
    print(f"  wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)", flush=True)


def channel(PF, g, sigma, B, seeds, decoding_type, q_bit, ps=0, pe=0, ss=0, se=0):
    wr = np.random.RandomState(seeds[0])
    nr = np.random.RandomState(seeds[1])
    X, Y = PF.create_mix_epoch(np.array([sigma]), wr, nr, B, g.N, g.N - g.M, g.z, [], True,
                               decoding_type, ps, pe, ss, se, q_bit, 20.0)
    return X, Y


def decoder_case(MF, PF, name, graph_name, z, sharing, decoding_type, q_bit, T, B, snr,
                 blocks=None, flat=None, target_node=0, fixed_iter=0, ps=0, pe=0, ss=0,
                 se=0, seeds=(2044, 1076), g=None, random_weights=None):
    print(f"[{name}]", flush=True)
    proto = load_proto(graph_name)
    if g is None:
        g = Graph(MF, proto, z, (snr,), ps, pe, ss, se)
    sigma = float(np.sqrt(1.0 / (2.0 * 10 ** (snr / 10.0) * g.rate)))
    if blocks is None:
        blocks = {}
        rng = np.random.RandomState(7)
        for kind, s in enumerate(sharing):
            if s <= 0:
                continue
            n_iter = T if s in (1, 2, 3) else fixed_iter + 1
            width = {1: g.E, 4: g.E, 3: 1}.get(s, g.M if kind < 2 else g.N)
            if random_weights is not None:
                lo, hi = random_weights
                blocks[kind] = rng.uniform(lo, hi, (n_iter, width)).astype(F32).astype(np.float64)
            else:
                blocks[kind] = np.full((n_iter, width), flat[kind])
    var_rows = var_rows_from_blocks(sharing, blocks, T, fixed_iter, g.M, g.N, g.E)
    X, Y = channel(PF, g, sigma, B, seeds, decoding_type, q_bit, ps, pe, ss, se)
    t0 = time.time()
    training_iter_start = fixed_iter
    net = run_graph(g, X, Y, sharing, decoding_type, q_bit, T, var_rows, target_node,
                    fixed_iter=fixed_iter, training_iter_start=training_iter_start)
    print(f"  reference graph B={B} T={T}: {time.time() - t0:.1f}s", flush=True)
    meta = dict(graph=graph_name, z=z, sharing=np.array(sharing, np.int32),
                decoding_type=decoding_type, q_bit=q_bit, T=T, B=B, snr=snr, sigma=sigma,
                target_node=target_node, fixed_iter=fixed_iter,
                punct=np.array([ps, pe], np.int32), short=np.array([ss, se], np.int32),
                seeds=np.array(seeds, np.int64))
    save_case(name, g, X, net, T, B, target_node, meta, var_rows, decoding_type)
    return g


def results_anchor(MF, PF, name="results_wman_303"):
    """compute_results (reference, unmodified) over a stand-in session."""
    print(f"[{name}]", flush=True)
    proto = load_proto("wman_N0576_R34_z24")
    z, T, B, sample_num = 24, 20, 120, 240
    snrs = np.array([2.0, 2.5, 3.0, 3.5, 4.0])
    g = Graph(MF, proto, z, snrs)
    sharing = [3, 0, 3]
    wf = os.path.join(REF, "Weights", "C0_wman_N0576_R34_z24_Opt_Weight_End20.txt")
    _, blocks = read_blocks(wf)
    blocks = {0: blocks[0], 2: blocks[2]}
    var_rows = var_rows_from_blocks(sharing, blocks, T, 0, g.M, g.N, g.E)

    class StandinSession:
        def run(self, fetches, feed_dict):
            net = run_graph(g, feed_dict["xa"], feed_dict["ya"], sharing, 2, 5, T, var_rows,
                            0, etha=feed_dict["etha"])
            if isinstance(fetches, list):
                return [net[k] for k in fetches]
            return net[fetches]

    net_dict = {k: k for k in ("xa", "ya", "etha", "learn_rate", "ya_output_all", "lossa")}
    wr = np.random.RandomState(2044)
    nr = np.random.RandomState(1076)
    t0 = time.time()
    Results, took = PF.compute_results(sample_num, [], [], g.sigma, wr, nr, B, 0, g.N, g.M, z,
                                       True, T, StandinSession(), net_dict, 0, 2, 0, 0, 0, 0,
                                       5, 20.0)
    print(f"  compute_results: {time.time() - t0:.1f}s\n  Results=\n{Results}", flush=True)
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, Results=Results, snr=snrs, sigma=g.sigma, sharing=np.array(sharing),
                        w0=var_rows[0], w2=var_rows[2], T=T, B=B, sample_num=sample_num,
                        seeds=np.array([2044, 1076]), graph="wman_N0576_R34_z24", z=z,
                        decoding_type=2, q_bit=5, rate=g.rate)
    print(f"  wrote {path}", flush=True)


def weight_loader_cases(MF):
    """Record weight_init's variables for the reference's own call sites."""
    print("[weights_reference_order]", flush=True)
    out = {}
    tmp = tempfile.mkdtemp()
    os.makedirs(os.path.join(tmp, "Weights"))
    cases = [
        # (tag, source file, out_filename, sharing, start, end, fixed_iter, M, N, E)
        ("post_wman", "Weights/C0_wman_N0576_R34_z24_Opt_Weight_End20.txt",
         "C0_wman_N0576_R34_z24", [3, 3, 3], 20, 30, 20, "wman_N0576_R34_z24"),
        ("base303_wman", "Weights/C0_wman_N0576_R34_z24_Opt_Weight_End20.txt",
         "C0_wman_N0576_R34_z24", [3, 0, 3], 20, 20, 0, "wman_N0576_R34_z24"),
        ("wifi50", "Results/WIFI/Weights_Iter50.txt", "wifi", [3, 3, 3], 50, 50, 0,
         "802_11n_N648_R56_z27"),
        ("g5_1024", "Results/5G/5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640_Weight_End50.txt",
         "g5", [2, 2, 2], 50, 50, 0, "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640"),
    ]
    cwd = os.getcwd()
    try:
        os.chdir(tmp)
        for tag, src, outname, sharing, start, end, fixed, gname in cases:
            proto = load_proto(gname)
            M, N = proto.shape
            E = int((proto != -1).sum())
            dst = os.path.join(tmp, "Weights", f"{outname}_Opt_Weight_End{start}.txt")
            shutil.copyfile(os.path.join(REF, src), dst)
            net = MF.weight_init({}, 0, outname, end, start, sharing, E, M, N, 0, 2, 1, 1, end,
                                 fixed)
            for key, val in net.items():
                out[f"{tag}/{key}"] = np.asarray(val, F32)
            out[f"{tag}/meta"] = np.array([start, end, fixed, M, N, E] + sharing, np.int64)
            out[f"{tag}/src"] = np.array(src)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp)
    path = os.path.join(HERE, "weights_reference_order.npz")
    np.savez_compressed(path, **out)
    print(f"  wrote {path} ({len(out)} arrays)", flush=True)


def channel_cases(PF):
    """create_mix_epoch outputs (reference) for the channel restatement test."""
    print("[channel]", flush=True)
    out = {}
    specs = [("wman_q5", 24, 24, 6, 2, 5, 0, 0, 0, 0, 2.5, 37),
             ("wman_ms", 24, 24, 6, 1, 5, 0, 0, 0, 0, 3.0, 5),
             ("g5_q5", 64, 20, 10, 2, 5, 1, 128, 513, 640, 2.0, 9),
             ("g5_sp", 64, 20, 10, 0, 5, 1, 128, 513, 640, 2.0, 4)]
    for tag, z, N, M, dt, q, ps, pe, ss, se, sigma, B in specs:
        wr = np.random.RandomState(2044)
        nr = np.random.RandomState(1076)
        X, Y = PF.create_mix_epoch(np.array([sigma / 4.0]), wr, nr, B, N, N - M, z, [], True,
                                   dt, ps, pe, ss, se, q, 20.0)
        X2, _ = PF.create_mix_epoch(np.array([sigma / 4.0, sigma / 3.0]), wr, nr, 7, N, N - M, z,
                                    [], True, dt, ps, pe, ss, se, q, 20.0)
        out[f"{tag}/X"] = X
        out[f"{tag}/X2"] = X2
        out[f"{tag}/Y"] = Y
        out[f"{tag}/spec"] = np.array([z, N, M, dt, q, ps, pe, ss, se, B], np.int64)
        out[f"{tag}/sigma"] = np.array([sigma / 4.0, sigma / 3.0])
        out[f"{tag}/next_noise"] = nr.normal(0, 1, 3)
        out[f"{tag}/next_word"] = wr.randint(0, 2, 3)
    path = os.path.join(HERE, "channel_reference.npz")
    np.savez_compressed(path, **out)
    print(f"  wrote {path}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*")
    args = ap.parse_args()
    MF, PF = import_reference()
    want = lambda n: not args.only or n in args.only   # noqa: E731

    wman_wf = os.path.join(REF, "Weights", "C0_wman_N0576_R34_z24_Opt_Weight_End20.txt")
    _, wman_blocks = read_blocks(wman_wf)
    if want("channel"):
        channel_cases(PF)
    if want("weights"):
        weight_loader_cases(MF)
    g_wman = None
    if want("wman_303_q5"):
        for snr in (2.0, 2.5, 3.5):
            g_wman = decoder_case(MF, PF, f"wman_303_q5_snr{snr}", "wman_N0576_R34_z24", 24,
                                  [3, 0, 3], 2, 5, 20, 24, snr,
                                  blocks={0: wman_blocks[0], 2: wman_blocks[2]}, g=g_wman)
    if want("wman_333_post"):
        # base+post cascade as one 30-iteration inference graph: rows 0..19 from the wman
        # file, 20..29 random (a stand-in for the post-decoder's trained rows).
        rng = np.random.RandomState(11)
        blocks = {k: np.concatenate([wman_blocks[k], rng.uniform(0.5, 1.2, (10, 1))])
                  for k in (0, 1, 2)}
        g_wman = decoder_case(MF, PF, "wman_333_post_snr2.0", "wman_N0576_R34_z24", 24,
                              [3, 3, 3], 2, 5, 30, 16, 2.0, blocks=blocks, g=g_wman)
    if want("wman_ms"):
        g_wman = decoder_case(MF, PF, "wman_303_ms_snr2.5", "wman_N0576_R34_z24", 24,
                              [3, 0, 3], 1, 5, 20, 16, 2.5,
                              blocks={0: wman_blocks[0], 2: wman_blocks[2]}, g=g_wman)
        g_wman = decoder_case(MF, PF, "wman_111_ms3_snr2.5", "wman_N0576_R34_z24", 24,
                              [1, 1, 2], 3, 5, 8, 8, 2.5, random_weights=(0.4, 1.1),
                              g=g_wman)
    if want("wman_qbits"):
        for q in (6, -5, 4, 3):
            g_wman = decoder_case(MF, PF, f"wman_222_q{q}".replace("-", "m"),
                                  "wman_N0576_R34_z24", 24, [2, 2, 2], 2, q, 10, 8, 2.5,
                                  random_weights=(0.5, 1.2), g=g_wman)
    if want("wman_sys_type4"):
        g_wman = decoder_case(MF, PF, "wman_403_sys_q5", "wman_N0576_R34_z24", 24, [4, 0, 3],
                              2, 5, 12, 8, 2.5, random_weights=(0.5, 1.2), target_node=18,
                              fixed_iter=4)
        g_wman = decoder_case(MF, PF, "wman_111_q5", "wman_N0576_R34_z24", 24, [1, 1, 2],
                              2, 5, 10, 8, 2.0, random_weights=(0.4, 1.2), g=g_wman)
    if want("sys_bitsliced"):
        # systematic output (main_Base.py:83-86: target_node = N - M) on configurations the
        # bit-sliced counters-only kernels serve: wman [3,0,3] q5 with the trained weights, and
        # 5G BG2 [2,2,2] with puncture / shortening (row / column weights, UCN)
        g_wman = decoder_case(MF, PF, "wman_303_sys_q5_snr2.5", "wman_N0576_R34_z24", 24,
                              [3, 0, 3], 2, 5, 20, 24, 2.5,
                              blocks={0: wman_blocks[0], 2: wman_blocks[2]}, target_node=18,
                              g=g_wman)
        _, gb = read_blocks(os.path.join(
            REF, "Results/5G/5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640_Weight_End50.txt"))
        decoder_case(MF, PF, "g5bg2_222_sys_q5_snr1.75",
                     "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640", 64, [2, 2, 2], 2, 5,
                     20, 12, 1.75, blocks=gb, target_node=10, ps=1, pe=128, ss=513, se=640)
    if want("wifi"):
        _, wb = read_blocks(os.path.join(REF, "Results/WIFI/Weights_Iter50.txt"))
        decoder_case(MF, PF, "wifi_333_q5_snr3.0", "802_11n_N648_R56_z27", 27, [3, 3, 3], 2,
                     5, 50, 12, 3.0, blocks=wb)
    if want("g5"):
        _, gb = read_blocks(os.path.join(
            REF, "Results/5G/5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640_Weight_End50.txt"))
        decoder_case(MF, PF, "g5bg2_222_q5_snr2.0",
                     "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640", 64, [2, 2, 2], 2, 5,
                     20, 8, 2.0, blocks=gb, ps=1, pe=128, ss=513, se=640)
    if want("g5bg1"):
        # 5G BG1 n2112: no weights ship for it; random per-iteration scalars
        # so beta changes every iteration (check degree 19, z = 72, puncture + shorten)
        decoder_case(MF, PF, "g5bg1_303_q5_snr3.0",
                     "5G_LDPC_R0.73_n_dec2304_n2112_k1536_z72_s1537_1584", 72, [3, 0, 3], 2,
                     5, 12, 8, 3.0, random_weights=(0.5, 1.2), ps=1, pe=144, ss=1537, se=1584)
    if want("g5bg1_t50"):
        # SURVEY 8d C5 as benchmarked: BG1 n2112, T = 50, flat [3,0,3] alpha 0.75 / beta 1 (no
        # trained weights ship for this code), puncture 1-144, shorten 1537-1584; 2.5 dB so
        # that some frames still fail after 50 iterations
        decoder_case(MF, PF, "g5bg1_303_flat_t50_snr2.5",
                     "5G_LDPC_R0.73_n_dec2304_n2112_k1536_z72_s1537_1584", 72, [3, 0, 3], 2,
                     5, 50, 6, 2.5, flat={0: 0.75, 2: 1.0}, ps=1, pe=144, ss=1537, se=1584)
    if want("z1"):
        decoder_case(MF, PF, "mackay_333_q5_snr2.5", "MACKAY_N96_K48", 1, [3, 3, 3], 2, 5, 20,
                     16, 2.5, flat={0: 0.75, 1: 0.5, 2: 1.0})
        decoder_case(MF, PF, "bch_303_q5_snr3.0", "BCH_63_51", 1, [3, 0, 3], 2, 5, 10, 16, 3.0,
                     flat={0: 0.75, 2: 1.0})
        decoder_case(MF, PF, "polar_303_ms_snr3.0", "Polar_64_48", 1, [3, 0, 3], 1, 5, 10, 16,
                     3.0, flat={0: 0.75, 2: 1.0})
        decoder_case(MF, PF, "polar_222_q5_snr3.0", "Polar_64_48", 1, [2, 2, 2], 2, 5, 10, 16,
                     3.0, random_weights=(0.5, 1.0))
    if want("sp"):
        # sum-product (decoding_type 0): float, checked with a documented tolerance
        g_wman = decoder_case(MF, PF, "wman_303_sp_snr2.5", "wman_N0576_R34_z24", 24,
                              [3, 0, 3], 0, 5, 10, 16, 2.5,
                              blocks={0: wman_blocks[0][:10], 2: wman_blocks[2][:10]}, g=g_wman)
        g_wman = decoder_case(MF, PF, "wman_333_sp_snr2.0", "wman_N0576_R34_z24", 24,
                              [3, 3, 3], 0, 5, 10, 8, 2.0,
                              blocks={k: wman_blocks[k][:10] for k in (0, 1, 2)}, g=g_wman)
        _, gb = read_blocks(os.path.join(
            REF, "Results/5G/5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640_Weight_End50.txt"))
        decoder_case(MF, PF, "g5bg2_222_sp_snr2.0",
                     "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640", 64, [2, 2, 2], 0, 5,
                     10, 8, 2.0, blocks={k: v[:10] for k, v in gb.items()}, ps=1, pe=128,
                     ss=513, se=640)
    if want("results"):
        results_anchor(MF, PF)


if __name__ == "__main__":
    main()
