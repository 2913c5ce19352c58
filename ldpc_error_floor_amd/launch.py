"""One process per GPU without a launcher: the rank plumbing shared by ``bench.py`` and
``tools/sweep_c5.py``.

The reference's concurrency is one process per GPU (``main_Base.py:14-15``).  A script run
with ``--gpus N > 1`` and no ``WORLD_SIZE`` in its environment calls ``launch_ranks`` before it
imports torch: ranks 0..N-1 of the same command start as fresh child processes with the
variables ``torch.distributed.run`` would set, the parent never initialises HIP and never
execs (on this pool an exec from a process that touched the GPU takes the machine down).
Under ``torch.distributed.run`` (``WORLD_SIZE`` set, 1 included) the script is one rank and
``init_rank_group`` joins the process group: ``nccl`` (RCCL over xGMI) with the rank's device,
or ``gloo`` to rehearse the multi-rank path on CPU.  Nothing here imports torch at module level.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

__all__ = ["free_port", "launch_ranks", "rank_info", "init_rank_group", "fail_hook"]


def free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(script: str, argv, n: int, tag: str = None, extra_env=None) -> int:
    """Start ranks 0..n-1 of ``python script argv`` as fresh child processes (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT as torch.distributed.run sets them) and wait.
    The children share this stdout.  Returns 0, or the status of the first rank that failed
    (the others are then terminated)."""
    tag = tag or os.path.basename(script)
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.update(extra_env or {})
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(script)] + list(argv),
                                      env=env))
    status = 0
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                print(f"{tag}: rank {procs.index(p)} exited with status {rc}; stopping the "
                      f"other ranks", file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return status


def fail_hook(rank: int, tag: str) -> None:
    """Test hook: ``LDPC_TEST_FAIL_RANK=r`` makes rank r exit with status 7 once its process
    group is up (the others then wait in their first collective), so a test can check that one
    failing rank stops the whole job with a non-zero status (``launch_ranks``)."""
    fr = os.environ.get("LDPC_TEST_FAIL_RANK")
    if fr is not None and int(fr) == rank:
        print(f"{tag}: rank {rank}: LDPC_TEST_FAIL_RANK, exiting with status 7", file=sys.stderr,
              flush=True)
        os._exit(7)


def rank_info():
    """(launched as a rank?, world, rank, local rank) from the environment."""
    on = "WORLD_SIZE" in os.environ
    return (on, int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_rank_group(backend: str, local: int):
    """The rank's device and process group.  ``nccl``: one GPU per rank (LOCAL_RANK), RCCL
    bound to it.  ``gloo``: CPU collectives; the device is ``cuda:LOCAL_RANK mod visible`` when
    a GPU is present (several ranks may share it), else the CPU.  Returns the torch device."""
    import torch
    import torch.distributed as dist
    launched, world, rank, _ = rank_info()
    if backend == "nccl":
        ndev = torch.cuda.device_count()
        if local >= ndev:
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {ndev} GPUs visible")
        dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        if launched:
            dist.init_process_group("nccl", device_id=dev)
        return dev
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    dev = torch.device("cuda", local % ndev) if ndev else torch.device("cpu")
    if ndev:
        torch.cuda.set_device(dev)
    if launched:
        dist.init_process_group(backend)
    return dev
