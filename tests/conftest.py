"""Shared pytest setup: markers, repo on sys.path, golden-fixture helpers."""
import glob
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = os.environ.get("LDPC_REFERENCE", "/root/reference")

# decoder fixtures produced by tests/golden/make_golden.py
DECODER_CASES = sorted(
    os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
    if not os.path.basename(p).startswith(("channel_", "weights_", "results_")))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP extension")


def load_case(name):
    """Fixture -> dict with graph, expanded weights and expected outputs."""
    from ldpc_error_floor_amd.code import TannerGraph
    from ldpc_error_floor_amd.weights import expand_weights
    d = dict(np.load(os.path.join(GOLDEN, name + ".npz")))
    z, T = int(d["z"]), int(d["T"])
    g = TannerGraph(d["proto"], z)
    rows = {k: d[f"w{k}"] for k in range(3) if f"w{k}" in d}
    W = expand_weights(tuple(int(x) for x in d["sharing"]), rows, T, g, int(d["fixed_iter"]))
    Nt = int(d["target_node"]) or g.N
    if "app_x2" in d:
        app = d["app_x2"].astype(np.float32) / 2
    else:
        app = d["app"]
    hard = np.unpackbits(d["hard_packed"], axis=-1)[..., :g.N * z]
    synd = np.unpackbits(d["synd_packed"], axis=-1)[..., :g.M * z]
    return dict(d=d, g=g, W=W, z=z, T=T, Nt=Nt, app=app, hard=hard, synd=synd,
                llr=d["llr"], dt=int(d["decoding_type"]), q=int(d["q_bit"]),
                exact=("app_x2" in d))


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def cuda_device():
    if not gpu_available():
        pytest.skip("no ROCm GPU")
    import torch
    return torch.device("cuda", 0)
