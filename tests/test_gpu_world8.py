"""The 8-rank job on the one GPU of the test box (GPU only): ``bench.py --gpus 8`` and
``tools/sweep_c5.py --gpus 8 --config C5`` start eight rank processes themselves
(``ldpc_error_floor_amd.launch``, no exec) with ``LDPC_*_BACKEND=gloo``, all on cuda:0 at a
small batch, exercising the launcher, the ports, the barriers, the counter all-reduce and the
per-rank checkpoint keys at the world size BASELINE configs[3] / configs[4] name (the driver's
8-GPU node runs the same path over RCCL).  World-8 counters equal world 1; the rank offsets
tile [0, 8B); one failing rank stops the job with a non-zero status."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "LDPC_TEST_FAIL_RANK")}
    env.update(kw)
    return env


def _bench(args, env):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    return r


def test_bench_world8_gloo_equals_world1(cuda_device):
    B, steps = 4096, 2
    base = ["--steps", str(steps), "--warmup", "1", "--no-cpu-baseline"]
    r8 = _bench(base + ["--gpus", "8", "--batch", str(B)], _env(LDPC_BENCH_BACKEND="gloo"))
    assert r8.returncode == 0, r8.stderr[-3000:]
    o8 = json.loads([l for l in r8.stdout.splitlines() if l.startswith("{")][-1])
    assert o8["n_gpus"] == 8 and o8["process_group"] == {"backend": "gloo", "world": 8}
    assert o8["counters"]["rank_offsets"] == [r * B for r in range(8)]
    assert o8["fer_at_snr"]["frames"] == 8 * B * steps
    r1 = _bench(base + ["--batch", str(8 * B)], _env())
    assert r1.returncode == 0, r1.stderr[-3000:]
    o1 = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][-1])
    assert o1["n_gpus"] == 1 and o1.get("process_group") is None
    keys = ("bit_err_last", "frame_err_last", "frame_err_all", "loss2")
    assert [o8["counters"][k] for k in keys] == [o1["counters"][k] for k in keys]
    assert o1["counters"]["frame_err_last"] > 0


def test_bench_world8_c4_gloo_equals_world1(cuda_device):
    """BASELINE configs[3]'s own workload (5G BG2 n1024, T=20, puncture / shorten, the batch
    sharded over 8 ranks): world-8 counters equal world 1 and the rank offsets tile [0, 8B)."""
    B, steps = 2048, 1
    base = ["--config", "C4", "--steps", str(steps), "--warmup", "1", "--no-cpu-baseline"]
    r8 = _bench(base + ["--gpus", "8", "--batch", str(B)], _env(LDPC_BENCH_BACKEND="gloo"))
    assert r8.returncode == 0, r8.stderr[-3000:]
    o8 = json.loads([l for l in r8.stdout.splitlines() if l.startswith("{")][-1])
    assert o8["n_gpus"] == 8 and o8["process_group"] == {"backend": "gloo", "world": 8}
    assert o8["counters"]["rank_offsets"] == [r * B for r in range(8)]
    r1 = _bench(base + ["--batch", str(8 * B)], _env())
    assert r1.returncode == 0, r1.stderr[-3000:]
    o1 = json.loads([l for l in r1.stdout.splitlines() if l.startswith("{")][-1])
    keys = ("bit_err_last", "frame_err_last", "frame_err_all", "loss2")
    assert [o8["counters"][k] for k in keys] == [o1["counters"][k] for k in keys]
    assert o1["counters"]["frame_err_last"] > 0


def test_bench_world8_rank_failure_stops_the_job(cuda_device):
    r = _bench(["--gpus", "8", "--batch", "4096", "--steps", "1", "--warmup", "1", "--no-cpu-baseline"],
               _env(LDPC_BENCH_BACKEND="gloo", LDPC_TEST_FAIL_RANK="5"))
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert "rank 5 exited with status 7" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_sweep_c5_world8_gloo_equals_world1(tmp_path):
    args = [sys.executable, os.path.join(ROOT, "tools", "sweep_c5.py"), "--config", "C5",
            "--snrs", "2.5,3.0", "--scan", "32768", "--deep", "32768", "--batch", "4096",
            "--deep-below", "0.9"]
    outs = {}
    for name, extra, env in (("w1", [], _env()),
                             ("w8", ["--gpus", "8"], _env(LDPC_SWEEP_BACKEND="gloo"))):
        out = str(tmp_path / name)
        r = subprocess.run(args + extra + ["--out", out], env=env, capture_output=True, text=True,
                           timeout=900, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        with open(os.path.join(out, "sweep_c5.json")) as f:
            outs[name] = json.load(f)
    assert outs["w1"]["process_group"] is None
    assert outs["w8"]["process_group"] == {"backend": "gloo", "world": 8}
    keys = ("snr_db", "codewords", "frame_err_last", "frame_err_any_iter", "bit_err_last")
    rows = lambda j: [[r[k] for k in keys] for r in j["scan"] + j["deep"]]  # noqa: E731
    assert rows(outs["w8"]) == rows(outs["w1"])
    assert outs["w1"]["scan"][0]["frame_err_last"] > 0 and outs["w1"]["deep"]
    for r in range(1, 8):
        assert os.path.exists(os.path.join(str(tmp_path / "w8"), f"ckpt_scan.json.rank{r}"))


def test_sweep_uncor_world2_file_equals_world1(tmp_path):
    """The multi-rank uncorrected-word collection on the GPU (gloo world 2 on one card, C2 at
    1.5 dB): the one merged Uncor file is byte-identical to world 1's, and the JSON rates give
    the collection sweep's throughput."""
    args = [sys.executable, os.path.join(ROOT, "tools", "sweep_c5.py"), "--config", "C2",
            "--deep-snrs", "1.5,2.0", "--deep", "20000", "--batch", "8192", "--uncor"]
    outs = {}
    for name, extra, env in (("w1", [], _env()),
                             ("w2", ["--gpus", "2"], _env(LDPC_SWEEP_BACKEND="gloo"))):
        out = str(tmp_path / name)
        r = subprocess.run(args + extra + ["--out", out], env=env, capture_output=True, text=True,
                           timeout=600, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        with open(os.path.join(out, "sweep_c2.json")) as f:
            outs[name] = json.load(f)
    w1 = open(os.path.join(str(tmp_path / "w1"), "Uncor_deep.txt"), "rb").read()
    w2 = open(os.path.join(str(tmp_path / "w2"), "Uncor_deep.txt"), "rb").read()
    n = sum(r["frame_err_any_iter"] for r in outs["w1"]["deep"])
    assert n > 0 and w1.count(b"\n") == n
    assert w2 == w1
