"""The on-GPU AWGN channel (ldpc_channel_awgn / ldpc_decode_awgn, csrc/ldpc_awgn.h) against
its CPU restatement oracle/philox_oracle.py (GPU only).  The oracle's Philox is pinned by the
Random123 known-answer vectors and its QMS level probabilities by the channel model
(tests/test_philox_oracle.py); this pins the device streams to it: QMS LLRs (the level
sampler) bit-exact for every q_bit and offset, float LLRs (Box-Muller) within a few ulps,
puncture / shorten exact, and every in-decoder generation (v5 prologue, the bit-sliced
kernels' prologue channel) equal to decoding the oracle's LLRs."""
import os

import numpy as np
import pytest

from conftest import ROOT
from oracle import nms_oracle
from oracle.philox_oracle import awgn_llr

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
@pytest.mark.parametrize("off", [123456, 123457])
def test_qms_channel_bit_exact(cuda_device, q, off):
    dec = _decoder(cuda_device, "wman_N0576_R34_z24", 24, 2, q)
    B, seed, sigma = 4099, (1 << 33) + 1076, 0.61
    got = dec.awgn(B, sigma, seed, offset=off).cpu().numpy()
    ref, _ = awgn_llr(B, dec.n_vars, sigma, seed, off, decoding_type=2, q_bit=q)
    assert np.array_equal(got, ref)


def test_qms_channel_puncture_shorten_bit_exact(cuda_device):
    dec = _decoder(cuda_device, G5, 64, 2, 5)
    B, off, seed, sigma = 1000, 77, 9, 0.7943282
    got = dec.awgn(B, sigma, seed, offset=off, punct=(1, 128), short=(513, 640)).cpu().numpy()
    ref, _ = awgn_llr(B, dec.n_vars, sigma, seed, off, decoding_type=2, q_bit=5, punct=(1, 128),
                      short=(513, 640))
    assert np.array_equal(got, ref)


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
    """In-kernel channel (the v5 prologue with an APP export, the bit-sliced kernels' byte
    channel for counters) == decoding the oracle's LLRs (flood and fused), and the oracle
    decoder agrees."""
    import torch
    from ldpc_error_floor_amd.code import CodeParams
    dec = _decoder(cuda_device, "wman_N0576_R34_z24", 24, 2, 5, T=20)
    sigma = float(CodeParams(dec.graph.proto, 24).sigma(2.0))
    B, off, seed = 2000, (1 << 20) + 2, 4242
    ref, _ = awgn_llr(B, dec.n_vars, sigma, seed, off, decoding_type=2, q_bit=5)
    ref_t = torch.from_numpy(ref).to(cuda_device)
    for k in ("fused", "flood"):
        want = dec.decode(ref_t, app=False, counters=True, flags=True, kernel=k, iter_wrong=True)
        got = dec.decode_awgn(B, sigma, seed, offset=off, counters=True, flags=True, kernel=k,
                              iter_wrong=True)
        for a, b in ((got.flags, want.flags), (got.counters, want.counters),
                     (got.iter_wrong, want.iter_wrong)):
            assert np.array_equal(a.cpu().numpy(), b.cpu().numpy()), k
        if k == "fused":
            assert dec.last_kernel().startswith("bsl[") and dec.last_kernel().endswith("+gen"), dec.last_kernel()
            assert dec.generates_channel_in_kernel(kernel=k)
        else:
            assert dec.last_kernel() == "flood" and not dec.generates_channel_in_kernel(kernel=k)
    # the v5 prologue channel (APP export)
    got = dec.decode_awgn(64, sigma, seed, offset=off + 5, app=True)
    assert dec.last_kernel().startswith("fused5[") and dec.last_kernel().endswith("+gen"), dec.last_kernel()
    assert dec.generates_channel_in_kernel(app=True)
    want = dec.decode(ref_t[5:69], app=True)
    assert np.array_equal(got.app.cpu().numpy(), want.app.cpu().numpy())
    W = dec.weights
    idx = np.arange(0, B, 31)[:64]
    o = nms_oracle.decode(ref[idx], dec.graph.proto, 24, W.alpha, W.alpha_ucn, W.beta, 20, 2, 5)
    app = dec.decode(ref_t[torch.from_numpy(idx).to(cuda_device)], app=True).app.cpu().numpy()
    assert np.array_equal(app, o["app"])


@pytest.mark.parametrize("config", ["C2", "C3", "C4", "C5"])
@pytest.mark.parametrize("off", [0, 3])
def test_byte_channel_equals_float_channel(config, off, cuda_device):
    """ldpc_decode_awgn's channel generated in the bit-sliced kernels' prologue (their Q8 build) gives
    the counters, frame flags and per-iteration frame errors of ldpc_channel_awgn's float LLRs
    decoded by the same kernel, on every SURVEY workload (shortened bits through the BIG
    marker on C4 / C5), ragged batch, aligned and unaligned offsets; LDPC_AWGN_Q8=0 is the
    float path through ldpc_decode_awgn (read once per process, so compared here through
    decode(awgn(...)))."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = bench.CONFIGS[config]
    proto, g, W, cp = bench.load_problem(config=config)
    dec = NMSDecoder(proto, cfg["z"], W, 2, 5, device=cuda_device)
    punct, short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    B, sigma = 8195, float(cp.sigma(cfg["snr"]))
    llr = dec.awgn(B, sigma, 17, offset=1000 + off, punct=punct, short=short)
    want = dec.decode(llr, app=False, counters=True, flags=True, iter_wrong=True)
    k_float = dec.last_kernel()
    got = dec.decode_awgn(B, sigma, 17, offset=1000 + off, punct=punct, short=short,
                          counters=True, flags=True, iter_wrong=True)
    # (the "+gen" marker: the channel was generated in the kernel's prologue, not read from HBM
    # -- a quiet fallback to the float path would decode the same LLRs to the same counters)
    assert dec.last_kernel() == k_float + "+gen" and k_float.startswith(("bsl[", "bsc[")), (k_float, dec.last_kernel())
    dec.short = short
    assert dec.generates_channel_in_kernel()
    for a, b in ((got.flags, want.flags), (got.counters, want.counters),
                 (got.iter_wrong, want.iter_wrong)):
        assert np.array_equal(a.cpu().numpy(), b.cpu().numpy())
    assert int(want.counters[1]) > 0


@pytest.mark.parametrize("off", [4096, 4097])
def test_qms_high_word_tie_bit_exact(cuda_device, off):
    """A uniform whose high word ties the lowest threshold (sigmas from
    test_philox_oracle.tie_sigmas): the device's low-word draw orders it like the oracle's
    64-bit comparison, in ldpc_channel_awgn's level sampler and in the v5 prologue's channel
    (aligned batches: awgn_levels4; unaligned: awgn_qms_elem) and in the bit-sliced kernels'
    prologue (awgn_levels4b, one or two quads per word)."""
    import torch
    from test_philox_oracle import tie_sigmas
    dec = _decoder(cuda_device, "wman_N0576_R34_z24", 24, 2, 5, T=2)
    seed = 7
    b, v, s0, s1 = tie_sigmas(dec.n_vars, seed, off & ~3, bmin=off & 3)
    b -= off & 3                              # the element's row in a batch starting at off
    for s, lv in ((s0, 0), (s1, 1)):
        B = 64
        got = dec.awgn(B, s, seed, offset=off).cpu().numpy()
        ref, _ = awgn_llr(B, dec.n_vars, s, seed, off, decoding_type=2, q_bit=5)
        assert ref[b, v] == (-7.5 if lv == 0 else -7.0)
        assert np.array_equal(got, ref)
        app = dec.decode_awgn(B, s, seed, offset=off, app=True).app.cpu().numpy()
        want = dec.decode(torch.from_numpy(ref).to(cuda_device), app=True).app.cpu().numpy()
        assert np.array_equal(app, want)
        # the bit-sliced kernel's in-prologue channel (counters-only): the same tie resolution
        got = dec.decode_awgn(B, s, seed, offset=off, counters=True, flags=True, iter_wrong=True)
        assert dec.last_kernel().startswith("bsl[") and dec.last_kernel().endswith("+gen"), dec.last_kernel()
        exp = dec.decode(torch.from_numpy(ref).to(cuda_device), app=False, counters=True, flags=True,
                         iter_wrong=True)
        for x, y in ((got.flags, exp.flags), (got.counters, exp.counters), (got.iter_wrong, exp.iter_wrong)):
            assert np.array_equal(x.cpu().numpy(), y.cpu().numpy())
