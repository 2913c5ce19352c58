"""tools/sweep_c5.py as a multi-rank job on CPU (gloo, world size 2, the oracle-backed stand-in
decoder): the configs[4] error-floor sweep's entry point splits each SNR point's codewords over
the ranks, and its output counters equal a single process's; a resume at another world size is
refused.  (The RCCL world-1 run of the same tool: tests/test_gpu_rccl.py.)"""
import json
import os
import sys

import pytest
import torch.multiprocessing as mp

from conftest import ROOT
from test_distributed import _free_port

sys.path.insert(0, os.path.join(ROOT, "tools"))

ARGS = ["--config", "C2", "--snrs", "2.0,3.5", "--scan", "40", "--deep", "24", "--batch", "8",
        "--deep-below", "0.5"]


def make_oracle_decoder(config, device, batch):
    import bench
    from _helpers import OracleDecoder
    proto, g, W, cp = bench.load_problem(config=config)
    return OracleDecoder(proto, bench.CONFIGS[config]["z"], W)


def _rank(rank, world, port, out, q):
    os.environ.update(WORLD_SIZE=str(world), RANK=str(rank), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), LDPC_SWEEP_BACKEND="gloo")
    import sweep_c5
    try:
        rc = sweep_c5.main(ARGS + ["--gpus", str(world), "--out", out],
                           make_decoder=make_oracle_decoder)
        q.put((rank, rc, ""))
    except Exception as e:                         # noqa: BLE001 - reported to the test
        q.put((rank, -1, f"{type(e).__name__}: {e}"))


def _run_ranks(world, out):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, out, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    return got


def _counters(out):
    with open(os.path.join(out, "sweep_c2.json")) as f:
        j = json.load(f)
    keys = ("snr_db", "codewords", "frame_err_last", "frame_err_any_iter", "bit_err_last")
    return j, [[r[k] for k in keys] for r in j["scan"] + j["deep"]]


def test_sweep_tool_world2_equals_world1(tmp_path, monkeypatch):
    import sweep_c5
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("LDPC_SWEEP_BACKEND", "gloo")
    one = str(tmp_path / "w1")
    assert sweep_c5.main(ARGS + ["--out", one], make_decoder=make_oracle_decoder) == 0
    j1, c1 = _counters(one)
    assert j1["n_gpus"] == 1 and j1["process_group"] is None
    assert j1["deep"] and c1[0][2] > 0              # errors at 2 dB, a deep stage ran

    two = str(tmp_path / "w2")
    got = _run_ranks(2, two)
    assert [g[1] for g in got] == [0, 0], got
    j2, c2 = _counters(two)
    assert j2["n_gpus"] == 2 and j2["process_group"] == {"backend": "gloo", "world": 2}
    assert c2 == c1
    assert os.path.exists(os.path.join(two, "ckpt_scan.json.rank1"))

    # the finished world-2 sweep resumes to the same counters at world 2 ...
    got = _run_ranks(2, two)
    assert [g[1] for g in got] == [0, 0], got
    assert _counters(two)[1] == c1
    # ... and is refused at world 1 (rank 0's checkpoint key holds world = 2)
    with pytest.raises(ValueError, match="checkpoint is for"):
        sweep_c5.main(ARGS + ["--out", two], make_decoder=make_oracle_decoder)
    # and a world-1 sweep's checkpoints are refused by a world-2 job, on both ranks
    got = _run_ranks(2, one)
    assert all(g[1] == -1 and "ValueError" in g[2] for g in got), got


def test_sweep_tool_world8_equals_world1(tmp_path, monkeypatch):
    """The world size configs[3] / configs[4] name (8 ranks, gloo on CPU): every SNR point's
    codewords split over eight ranks give the counters of one process, and each rank keeps its
    own checkpoint."""
    import sweep_c5
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("LDPC_SWEEP_BACKEND", "gloo")
    one = str(tmp_path / "w1")
    assert sweep_c5.main(ARGS + ["--out", one], make_decoder=make_oracle_decoder) == 0
    _, c1 = _counters(one)
    eight = str(tmp_path / "w8")
    got = _run_ranks(8, eight)
    assert [g[1] for g in got] == [0] * 8, got
    j8, c8 = _counters(eight)
    assert j8["n_gpus"] == 8 and j8["process_group"] == {"backend": "gloo", "world": 8}
    assert c8 == c1
    for r in range(1, 8):
        assert os.path.exists(os.path.join(eight, f"ckpt_scan.json.rank{r}"))
