"""The fused float-mode kernels (csrc/ldpc_ffl.hip: min-sum fp32, min-sum without the nudge,
QMS q = 6, and the sum-product kernel k_ffs) that serve counters-only decodes (GPU only).  Its arithmetic is the flood kernel's
operation for operation, so counters and per-frame flags must equal flood's bit for bit (flood's
APP is pinned to the reference fixtures in test_gpu_parity.py): wman with trained [3,0,3] and
UCN [3,3,3] weights, 5G BG2 with puncture / shortening, ragged batches."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")


def _dec(device, cfg, dt, q, T=None, ucn=False):
    import bench
    from ldpc_error_floor_amd.code import TannerGraph, load_base_graph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights, read_weight_file
    c = bench.CONFIGS[cfg]
    if cfg == "C2" and ucn:
        proto = load_base_graph(os.path.join(DATA, "BaseGraph", c["graph"] + ".txt"))
        g = TannerGraph(proto, c["z"])
        wf = read_weight_file(os.path.join(DATA, c["weights"]))
        W = expand_weights((3, 3, 3), dict(wf.blocks), T or 20, g)
        cp = bench.load_problem(T=T, config=cfg)[3]
    else:
        proto, g, W, cp = bench.load_problem(T=T, config=cfg)
    # (sum-product runs the fused kernel only when asked for: AUTO keeps it on flood)
    dec = NMSDecoder(proto, c["z"], W, dt, q, device=device, kernel="fused" if dt == 0 else "auto")
    dec.punct = c.get("punct", (0, 0))
    dec.short = c.get("short", (0, 0))
    return dec, cp, c


@pytest.mark.parametrize("cfg,dt,q,ucn,B,snr", [
    ("C2", 1, 5, False, 3001, 2.0), ("C2", 3, 5, False, 777, 2.0), ("C2", 2, 6, False, 3001, 2.0),
    ("C2", 1, 5, True, 2049, 2.25), ("C4", 1, 5, True, 1000, 1.25), ("C4", 3, 5, True, 257, 1.25),
    ("C2", 1, 5, False, 40000, 2.5),
    # sum-product (decoding_type 0): flood's tanh / atanh arithmetic on per-edge LDS messages
    ("C2", 0, 5, False, 3001, 2.0), ("C2", 0, 5, True, 2049, 2.25), ("C4", 0, 5, True, 1000, 1.0),
    ("C3", 0, 5, True, 513, 3.0), ("C5", 0, 5, False, 300, 2.5)])
def test_ffl_equals_flood(cuda_device, cfg, dt, q, ucn, B, snr):
    dec, cp, c = _dec(cuda_device, cfg, dt, q, ucn=ucn)
    name = dec.kernel_info()[1]
    assert name.startswith("ffl[sp," if dt == 0 else "ffl[cw"), name
    llr = dec.awgn(B, float(cp.sigma(snr)), seed=13, offset=5)
    out = {}
    for k in ("flood", "fused"):
        r = dec.decode(llr, app=False, counters=True, flags=True, kernel=k)
        out[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy())
    assert np.array_equal(out["fused"][0], out["flood"][0]), (out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    assert 0 < out["fused"][0][1] < B


def test_ffl_app_export_stays_on_flood(cuda_device):
    """An APP / bit export in a float mode runs flood under AUTO; FUSED refuses it."""
    dec, cp, c = _dec(cuda_device, "C2", 1, 5)
    llr = dec.awgn(64, float(cp.sigma(2.0)), seed=1)
    r = dec.decode(llr, app=True, counters=True)
    f = dec.decode(llr, app=False, counters=True)
    assert np.array_equal(r.counters.cpu().numpy(), f.counters.cpu().numpy())
    with pytest.raises(RuntimeError):
        dec.decode(llr, app=True, kernel="fused")


def test_ffl_decode_awgn_matches_channel_then_decode(cuda_device):
    dec, cp, c = _dec(cuda_device, "C4", 1, 5)
    sigma = float(cp.sigma(1.25))
    a = dec.decode_awgn(2000, sigma, seed=3, offset=11, counters=True, flags=True)
    llr = dec.awgn(2000, sigma, seed=3, offset=11)
    b = dec.decode(llr, app=False, counters=True, flags=True, kernel="flood")
    assert np.array_equal(a.counters.cpu().numpy(), b.counters.cpu().numpy())
    assert np.array_equal(a.flags.cpu().numpy(), b.flags.cpu().numpy())


def test_ffl_refuses_per_edge_weights(cuda_device):
    """Per-edge CN weights (sharing 1) have no compressed record: AUTO decodes them with flood."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights
    proto, g, _, cp = bench.load_problem(T=8, config="C2")
    rng = np.random.RandomState(2)
    W = expand_weights((1, 0, 3), {0: rng.uniform(0.5, 1.0, (8, g.E)), 2: np.ones((8, 1))}, 8, g)
    dec = NMSDecoder(proto, 24, W, 1, 5, device=cuda_device)
    assert dec.kernel_info()[1] == "flood", dec.kernel_info()
    llr = dec.awgn(500, float(cp.sigma(2.0)), seed=4)
    a = dec.decode(llr, app=False, counters=True)
    b = dec.decode(llr, app=False, counters=True, kernel="flood")
    assert np.array_equal(a.counters.cpu().numpy(), b.counters.cpu().numpy())


def test_ffl_sp_per_edge_weights(cuda_device):
    """Sum-product keeps every edge's message, so per-edge CN weights (sharing 1) stay on the
    fused kernel and equal flood's counters."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights
    proto, g, _, cp = bench.load_problem(T=8, config="C2")
    rng = np.random.RandomState(2)
    W = expand_weights((1, 0, 3), {0: rng.uniform(0.5, 1.0, (8, g.E)), 2: np.ones((8, 1))}, 8, g)
    dec = NMSDecoder(proto, 24, W, 0, 5, device=cuda_device, kernel="fused")
    assert dec.kernel_info()[1].startswith("ffl[sp,"), dec.kernel_info()
    assert NMSDecoder(proto, 24, W, 0, 5, device=cuda_device).kernel_info()[1] == "flood"
    llr = dec.awgn(1500, float(cp.sigma(2.0)), seed=4)
    a = dec.decode(llr, app=False, counters=True, flags=True)
    b = dec.decode(llr, app=False, counters=True, flags=True, kernel="flood")
    assert np.array_equal(a.counters.cpu().numpy(), b.counters.cpu().numpy())
    assert np.array_equal(a.flags.cpu().numpy(), b.flags.cpu().numpy())
