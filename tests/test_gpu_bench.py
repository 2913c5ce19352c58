"""bench.py's multi-rank path (GPU only): ``bench.py --gpus 2`` started without a launcher
spawns its two ranks itself; with LDPC_BENCH_BACKEND=gloo both share the one GPU of the test
box.  The all-reduced counters must equal two single-process decodes of the rank slices
(global Philox offsets 0 and B), and the JSON line must report the whole job."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_spawns_ranks_and_reduces(cuda_device):
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    B, steps = 4096, 2
    env = dict(os.environ, LDPC_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch",
                        str(B), "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2"
    assert out["fer_at_snr"]["frames"] == 2 * B * steps
    assert out["counters"]["rank_offsets"] == [0, B]
    cfg = bench.CONFIGS["C2"]
    proto, g, W, cp = bench.load_problem(config="C2")
    dec = NMSDecoder(proto, 24, W, 2, 5, device=cuda_device)
    cnt = torch.zeros(4, dtype=torch.int64, device=cuda_device)
    for off in (0, B):
        llr = dec.awgn(B, float(cp.sigma(cfg["snr"])), seed=1076, offset=off)
        dec.decode(llr, T=cfg["T"], app=False, counters=cnt)
    want = [steps * v for v in cnt.cpu().tolist()]
    c = out["counters"]
    assert [c["bit_err_last"], c["frame_err_last"], c["frame_err_all"], c["loss2"]] == want


def test_bench_rank_failure_propagates():
    """A rank that fails makes the launcher exit non-zero (and stops the other rank)."""
    env = dict(os.environ, LDPC_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--config", "C2", "--iters", "999", "--batch", "256", "--steps", "1",
                        "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode != 0
    assert "exited with status" in r.stderr
