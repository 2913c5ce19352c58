"""The on-GPU AWGN channel (ldpc_channel_awgn / ldpc_decode_awgn, csrc/ldpc_awgn.h) against
its CPU restatement oracle/philox_oracle.py (GPU only).  The oracle's Philox is pinned by the
Random123 known-answer vectors (tests/test_philox_oracle.py); this pins the device stream to
it: quantized LLRs bit-exact (except within ulps of a grid rounding boundary, where the device
logf / sincospif may round the other way), float LLRs within a few ulps, puncture / shorten
exact, and the in-decoder generation equal to decoding the oracle's LLRs."""
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import nms_oracle
from oracle.philox_oracle import awgn_llr, near_boundary

pytestmark = pytest.mark.gpu
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")
G5 = "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640"


def _decoder(device, graph, z, dt, q, T=8):
    from ldpc_error_floor_amd.code import TannerGraph, load_base_graph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import flat_weights
    proto = load_base_graph(os.path.join(DATA, "BaseGraph", graph + ".txt"))
    return NMSDecoder(proto, z, flat_weights(TannerGraph(proto, z), T, 0.75), dt, q,
                      device=device)


@pytest.mark.parametrize("q", [5, 6, -5, 4, 3])
def test_qms_channel_bit_exact(cuda_device, q):
    dec = _decoder(cuda_device, "wman_N0576_R34_z24", 24, 2, q)
    B, off, seed, sigma = 4096, 123457, (1 << 33) + 1076, 0.61
    got = dec.awgn(B, sigma, seed, offset=off).cpu().numpy()
    ref, raw = awgn_llr(B, dec.n_vars, sigma, seed, off, decoding_type=2, q_bit=q)
    edge = near_boundary(raw, q)
    assert edge.mean() < 1e-3
    assert np.array_equal(got[~edge], ref[~edge])
    # at a boundary the two roundings are adjacent grid values
    step = {6: 1.0, 5: 0.5, -5: 1.0, 4: 1.0, 3: 2.0}[q]
    assert np.all(np.abs(got[edge] - ref[edge]) <= step)


@pytest.mark.parametrize("dt", [1, 0])
def test_float_channel_within_ulps_puncture_shorten(cuda_device, dt):
    dec = _decoder(cuda_device, G5, 64, dt, 5)
    B, off, seed, sigma = 1024, 77, 9, 0.7943282
    got = dec.awgn(B, sigma, seed, offset=off, punct=(1, 128), short=(513, 640)).cpu().numpy()
    ref, raw = awgn_llr(B, dec.n_vars, sigma, seed, off, decoding_type=dt, punct=(1, 128),
                        short=(513, 640))
    assert np.array_equal(got[:, :128], ref[:, :128])          # 0 (MS) / 0.001 (SP)
    assert np.array_equal(got[:, 512:640], ref[:, 512:640])    # -clip_LLR
    body = np.r_[128:512, 640:1280]
    # Box-Muller through the device logf / sincospif: a few fp32 ulps of |sigma n| in the LLR
    tol = 8 * np.spacing(np.abs(raw[:, body]) + np.float32(2 / sigma ** 2)) + 1e-6
    assert np.all(np.abs(got[:, body] - ref[:, body]) <= tol)


def test_decode_awgn_equals_decoding_oracle_llrs(cuda_device):
    """In-kernel channel (fused v5 prologue) == decoding the oracle's LLRs (flood and fused),
    and the oracle decoder agrees, on codewords away from grid boundaries."""
    import torch
    from ldpc_error_floor_amd.code import CodeParams
    dec = _decoder(cuda_device, "wman_N0576_R34_z24", 24, 2, 5, T=20)
    sigma = float(CodeParams(dec.graph.proto, 24).sigma(2.0))
    B, off, seed = 2000, 1 << 20, 4242
    ref, raw = awgn_llr(B, dec.n_vars, sigma, seed, off, decoding_type=2, q_bit=5)
    clean = ~near_boundary(raw, 5).any(axis=1)
    assert clean.mean() > 0.5
    ref_t = torch.from_numpy(ref).to(cuda_device)
    for k in ("fused", "flood"):
        want = dec.decode(ref_t, app=False, counters=True, flags=True, kernel=k)
        got = dec.decode_awgn(B, sigma, seed, offset=off, counters=True, flags=True, kernel=k)
        f_got, f_want = got.flags.cpu().numpy(), want.flags.cpu().numpy()
        assert np.array_equal(f_got[clean], f_want[clean]), k
    W = dec.weights
    idx = np.flatnonzero(clean)[:64]
    o = nms_oracle.decode(ref[idx], dec.graph.proto, 24, W.alpha, W.alpha_ucn, W.beta, 20, 2, 5)
    app = dec.decode(ref_t[torch.from_numpy(idx).to(cuda_device)], app=True).app.cpu().numpy()
    assert np.array_equal(app, o["app"])
