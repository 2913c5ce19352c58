"""The RCCL code path on the one GPU of the test box (GPU only).

bench.py and fer_sweep initialise a process group whenever they run as a rank (WORLD_SIZE set,
1 included), so a world of one executes the same ``init_process_group("nccl", device_id=...)``,
``barrier(device_ids=...)`` and device-tensor ``all_reduce`` the 8-GPU job runs; the reference's
own concurrency is one process per GPU (``main_Base.py:14-15``).  Both run in child processes
(fresh HIP state, bounded by a timeout) and must give the counters of the same work done without
any process group."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_env():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0", LOCAL_WORLD_SIZE="1",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
    env.pop("LDPC_BENCH_BACKEND", None)          # the default backend: nccl (RCCL)
    env.pop("LDPC_SWEEP_BACKEND", None)
    return env


def test_bench_world1_over_rccl(cuda_device):
    import torch
    sys.path.insert(0, ROOT)
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    B, steps = 8192, 2
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--batch", str(B),
                        "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline"],
                       env=_rank_env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["process_group"] == {"backend": "nccl", "world": 1}
    assert out["n_gpus"] == 1 and out["fer_at_snr"]["frames"] == B * steps
    cfg = bench.CONFIGS["C2"]
    proto, g, W, cp = bench.load_problem(config="C2")
    dec = NMSDecoder(proto, 24, W, 2, 5, device=cuda_device)
    cnt = torch.zeros(4, dtype=torch.int64, device=cuda_device)
    llr = dec.awgn(B, float(cp.sigma(cfg["snr"])), seed=1076, offset=0)
    dec.decode(llr, T=cfg["T"], app=False, counters=cnt)
    c = out["counters"]
    assert [c["bit_err_last"], c["frame_err_last"], c["frame_err_all"], c["loss2"]] == \
        [steps * v for v in cnt.cpu().tolist()]


SWEEP = r"""
import json, os, sys
sys.path.insert(0, os.environ["LDPC_ROOT"])
import torch, torch.distributed as dist
import bench
from ldpc_error_floor_amd.decoder import NMSDecoder
from ldpc_error_floor_amd.fer import fer_sweep
proto, g, W, cp = bench.load_problem(config="C2")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dec = NMSDecoder(proto, 24, W, 2, 5, device=dev)
sig = [float(cp.sigma(2.0)), float(cp.sigma(2.75))]
plain = fer_sweep(dec, sig, 20000, 4096, seed=5)
dist.init_process_group("nccl", device_id=dev)
grouped = fer_sweep(dec, sig, 20000, 4096, seed=5)
dist.barrier(device_ids=[0])
be = dist.get_backend()
dist.destroy_process_group()
f = lambda res: [[r.bit_err_last, r.frame_err_last, r.frame_err_all, r.loss2] for r in res]
print(json.dumps({"backend": be, "plain": f(plain), "grouped": f(grouped)}))
"""


def test_fer_sweep_over_rccl_group(cuda_device):
    env = dict(_rank_env(), LDPC_ROOT=ROOT)
    r = subprocess.run([sys.executable, "-c", SWEEP], env=env, capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["backend"] == "nccl"
    assert out["grouped"] == out["plain"]
    assert out["plain"][0][1] > 0


def test_sweep_tool_world1_over_rccl(tmp_path):
    """tools/sweep_c5.py (the configs[4] multi-GPU sweep entry point) as an RCCL world-1 rank
    gives the counters of the same sweep run without a process group."""
    args = [sys.executable, os.path.join(ROOT, "tools", "sweep_c5.py"), "--config", "C2",
            "--snrs", "2.0,4.0", "--scan", "65536", "--deep", "98304", "--batch", "32768",
            "--deep-below", "0.5"]
    plain_env = {k: v for k, v in os.environ.items()
                 if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LDPC_SWEEP_BACKEND")}
    outs = {}
    for name, env in (("plain", plain_env), ("rccl", _rank_env())):
        out = str(tmp_path / name)
        r = subprocess.run(args + ["--out", out], env=env, capture_output=True, text=True,
                           timeout=300, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        with open(os.path.join(out, "sweep_c2.json")) as f:
            outs[name] = json.load(f)
    assert outs["plain"]["process_group"] is None
    assert outs["rccl"]["process_group"] == {"backend": "nccl", "world": 1}
    strip = lambda j: [{k: v for k, v in r.items()} for r in j["scan"] + j["deep"]]  # noqa: E731
    assert strip(outs["rccl"]) == strip(outs["plain"])
    assert outs["plain"]["scan"][0]["frame_err_last"] > 0 and outs["plain"]["deep"]
