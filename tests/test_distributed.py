"""Multi-process FER sweep on CPU (gloo, world_size 2): every rank decodes a disjoint
contiguous range of the global codeword stream and ONE all_reduce(SUM) of the counter block
gives the same totals as a single process."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import GOLDEN, ROOT
from ldpc_error_floor_amd.fer import fer_sweep, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_decoder():
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _helpers import OracleDecoder
    from ldpc_error_floor_amd.code import TannerGraph, load_base_graph
    from ldpc_error_floor_amd.weights import expand_weights
    d = np.load(os.path.join(GOLDEN, "results_wman_303.npz"))
    proto = load_base_graph(os.path.join(ROOT, "ldpc_error_floor_amd", "data", "BaseGraph",
                                         "wman_N0576_R34_z24.txt"))
    W = expand_weights((3, 0, 3), {0: d["w0"], 2: d["w2"]}, 20, TannerGraph(proto, 24))
    return OracleDecoder(proto, 24, W)


SIGMAS = [0.7943282, 0.65]
N_CW, BATCH = 45, 8


def _worker(rank, world, port, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        res = fer_sweep(_make_decoder(), SIGMAS, N_CW, BATCH, seed=1076)
        q.put((rank, [(c.bit_err_last, c.frame_err_last, c.frame_err_all, c.loss2) for c in res]))
    finally:
        dist.destroy_process_group()


def _uncor_worker(rank, world, port, q, path, ck, resume):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        res = fer_sweep(_make_decoder(), SIGMAS, N_CW, BATCH, seed=1076, uncor_path=path,
                        checkpoint=ck, resume=resume, checkpoint_every=2)
        q.put((rank, [c.frame_err_all for c in res]))
    finally:
        dist.destroy_process_group()


def _run_world(world, target, extra):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + extra) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_gloo_world2_uncorrected_file_equals_single_process(tmp_path):
    """The multi-rank uncorrected-word collection ends in ONE file, byte-identical to the
    single-process sweep's (global codeword order, SNR point by point): each rank writes
    <path>.rank<r> with per-point marks, rank 0 merges after the all-reduce
    (Print_Functions.py:120-126 writes the file main_Post.py reads, Main_Functions.py:529-532).
    Rows already in the file stay in front (the reference appends); a resume of the finished
    sweep merges again to the same bytes."""
    single = tmp_path / "single.txt"
    res1 = fer_sweep(_make_decoder(), SIGMAS, N_CW, BATCH, seed=1076, uncor_path=str(single))
    assert res1[0].frame_err_all > 0
    path = tmp_path / "Uncor.txt"
    path.write_bytes(b"earlier\trow\n")
    ck = str(tmp_path / "u.ckpt")
    got = _run_world(2, _uncor_worker, (str(path), ck, False))
    assert got[0] == got[1] == [c.frame_err_all for c in res1]
    assert path.read_bytes() == b"earlier\trow\n" + single.read_bytes()
    assert os.path.exists(f"{path}.rank1")
    # a resumed finished sweep: the same file, not the rows twice
    _run_world(2, _uncor_worker, (str(path), ck, True))
    assert path.read_bytes() == b"earlier\trow\n" + single.read_bytes()
    rows = np.loadtxt(path, delimiter="\t", ndmin=2, skiprows=1)
    assert rows.shape == (sum(c.frame_err_all for c in res1), 3 + 576)


def test_shard_range_partitions():
    for total in (0, 1, 7, 45, 1 << 20):
        for world in (1, 2, 3, 8):
            parts = [shard_range(total, r, world) for r in range(world)]
            assert parts[0][0] == 0 and parts[-1][1] == total
            assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))


def test_gloo_world2_equals_single_process():
    single = [(c.bit_err_last, c.frame_err_last, c.frame_err_all, c.loss2)
              for c in fer_sweep(_make_decoder(), SIGMAS, N_CW, BATCH, seed=1076)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0] == got[1] == single
    assert single[0][1] > 0           # the low-SNR point has frame errors


def test_sweep_collects_uncorrected_frames(tmp_path):
    """fer_sweep(uncor_path=...) appends exactly the frames wrong at every iteration, in the
    Uncor.txt row format, in stream order (host logic; the GPU compaction is tested on GPU)."""
    from ldpc_error_floor_amd.channel import write_uncor_file
    dec = _make_decoder()
    path = tmp_path / "Uncor.txt"
    res = fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=1076, uncor_path=str(path))
    rows = np.loadtxt(path, delimiter="\t", ndmin=2)
    assert rows.shape == (res[0].frame_err_all, 3 + dec.n_vars)
    # the same frames through the reference-format writer on host LLRs
    expect = tmp_path / "expect.txt"
    for pos in range(0, N_CW, BATCH):
        b = min(BATCH, N_CW - pos)
        llr = dec.awgn(b, SIGMAS[0], 1076, offset=pos)
        flags = torch.zeros(b, dtype=torch.uint8)
        dec.decode(llr, app=False, flags=flags)
        uncor = (flags.numpy() & 1).astype(np.float64)
        if uncor.sum():
            write_uncor_file(uncor, llr.numpy().reshape(b, dec.N, dec.z), dec.n_vars, str(expect))
    assert path.read_text() == expect.read_text()


def test_bench_launcher_spawns_and_propagates_failure():
    """bench.py --gpus 2 without a launcher starts two rank processes itself (RANK /
    WORLD_SIZE / MASTER_* set, no exec) and exits non-zero when a rank fails — here both fail
    for want of a GPU.  (The GPU run of the same path: tests/test_gpu_bench.py.)"""
    import subprocess
    import sys
    if torch.cuda.is_available():
        pytest.skip("GPU present: covered by test_gpu_bench.py")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--no-cpu-baseline", "--batch", "256"], env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0
    assert "rank 0: LOCAL_RANK 0" in r.stderr and "rank 1: LOCAL_RANK 1" in r.stderr
    assert "exited with status" in r.stderr


def _session_worker(rank, world, port, q, shard=True, seed_per_rank=False):
    """One rank of the parity-mode FER loop: the reference's compute_results over a Session
    that decodes this rank's slice of every host batch and gathers the rest (gloo).
    ``shard=False``: a plain Session under the same process group (no communication);
    ``seed_per_rank``: rank r draws its noise from seed 1076 + r (a sharded Session refuses)."""
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        from ldpc_error_floor_amd import fer
        from ldpc_error_floor_amd.session import Session, make_net_dict
        d = np.load(os.path.join(GOLDEN, "results_wman_303.npz"))
        dec = _make_decoder()
        calls = []
        inner = dec.decode

        def spy(llr, **kw):                       # record the slice sizes this rank decodes
            calls.append(np.asarray(llr).shape[0])
            return inner(llr, **kw)
        dec.decode = spy
        sess = Session(dec, batch_size=int(d["B"]), shard=shard)
        wr = np.random.RandomState(2044)
        nr = np.random.RandomState(1076 + (rank if seed_per_rank else 0))
        try:
            Results, _ = fer.compute_results(int(d["sample_num"]), [], [], d["sigma"], wr, nr,
                                             int(d["B"]), 0, 24, 6, 24, True, 20, sess,
                                             make_net_dict(20), 0, 2, 0, 0, 0, 0, 5, 20.0)
        except RuntimeError as e:
            q.put((rank, str(e), calls))
            return
        q.put((rank, Results.tolist(), calls))
    finally:
        dist.destroy_process_group()


def _run_session_ranks(**kw):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_session_worker, args=(r, 2, port, q), kwargs=kw)
             for r in range(2)]
    for p in procs:
        p.start()
    got = dict((r, (res, calls)) for r, res, calls in (q.get(timeout=600) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return got


def test_session_parity_mode_sharded_over_ranks():
    """SURVEY §8 e parity mode: host-generated LLRs sliced by rank.  Two gloo ranks each decode
    half of every 120-codeword batch and all_gather the APP; both reproduce the reference's own
    compute_results Results (tests/golden/results_wman_303.npz) exactly."""
    d = np.load(os.path.join(GOLDEN, "results_wman_303.npz"))
    got = _run_session_ranks(shard=True)
    B = int(d["B"])
    for r in (0, 1):
        np.testing.assert_array_equal(np.asarray(got[r][0], np.float32), d["Results"])
        b0, b1 = shard_range(B, r, 2)
        assert set(got[r][1]) == {b1 - b0}         # only its own slice, every call


def test_session_unsharded_under_process_group_decodes_whole_batches():
    """Without shard=True a Session under an initialised process group never communicates:
    each rank decodes its whole batches (the reference's one-process-per-GPU model,
    main_Base.py:14-15), here with a different noise seed per rank."""
    d = np.load(os.path.join(GOLDEN, "results_wman_303.npz"))
    got = _run_session_ranks(shard=False, seed_per_rank=True)
    B = int(d["B"])
    np.testing.assert_array_equal(np.asarray(got[0][0], np.float32), d["Results"])
    assert not np.array_equal(np.asarray(got[1][0], np.float32), d["Results"])
    for r in (0, 1):
        assert set(got[r][1]) == {B}


def test_session_sharded_refuses_different_batches():
    """A sharded Session whose ranks feed different xa raises on every rank instead of
    returning APP rows other ranks decoded from their own batches."""
    got = _run_session_ranks(shard=True, seed_per_rank=True)
    for r in (0, 1):
        assert isinstance(got[r][0], str) and "different xa" in got[r][0]
        assert got[r][1] == []
