"""Correctness at the benchmark's batch size (GPU only): B = 2^20 codewords in one launch for
C2 (wman, T=20, bit-sliced bsl kernel) and C5 (5G BG1 n2112, T=50, compressed bsc kernel: B * n_vars = 2.4e9 > 2^31, so every index into the
LLR block must be 64-bit).  The fused and flood kernels (both parity-pinned on the reference
fixtures) must agree frame by frame, and the first and last codewords of the batch, decoded on
their own, must match the oracle and the big launch's per-frame flags."""
import numpy as np
import pytest

from oracle import nms_oracle

pytestmark = pytest.mark.gpu
B = 1 << 20


@pytest.mark.parametrize("config,lpc", [("C2", "2"), ("C2", "4"), ("C5", "")])
def test_full_batch_kernels_agree_and_match_oracle(cuda_device, config, lpc, monkeypatch):
    if lpc:
        monkeypatch.setenv("LDPC_BS_LPC", lpc)
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = bench.CONFIGS[config]
    proto, g, W, cp = bench.load_problem(config=config)
    T, z = cfg["T"], cfg["z"]
    punct, short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    # an SNR where a visible share of frames fails, so the flags carry information
    snr = {"C2": 2.5, "C5": 2.5}[config]
    sigma = float(cp.sigma(snr))
    dec = NMSDecoder(proto, z, W, 2, 5, device=cuda_device, B_max=B)
    # counters-only decodes: the bit-sliced kernels (bsl for C2, the compressed bsc for C5)
    assert dec.kernel_info(T)[1].startswith({"C2": "bsl[", "C5": "bsc["}[config]), dec.kernel_info(T)
    llr = dec.awgn(B, sigma, seed=31, punct=punct, short=short)
    res = {}
    for k in ("fused", "flood"):
        r = dec.decode(llr, T=T, app=False, counters=True, flags=True, kernel=k)
        res[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy())
        torch.cuda.synchronize()
    assert np.array_equal(res["fused"][0], res["flood"][0])
    assert np.array_equal(res["fused"][1], res["flood"][1])
    cnt, flags = res["fused"]
    assert 0 < cnt[1] < B
    assert cnt[1] == int(((flags >> 1) & 1).sum()) and cnt[2] == int((flags & 1).sum())
    # in-decoder channel over the same global stream: same counters and flags
    r = dec.decode_awgn(B, sigma, 31, punct=punct, short=short, T=T, counters=True, flags=True)
    assert np.array_equal(r.counters.cpu().numpy(), cnt)
    assert np.array_equal(r.flags.cpu().numpy(), flags)
    # both ends of the batch against the oracle
    n = 96 if config == "C2" else 48
    for lo in (0, B - n):
        x = llr[lo:lo + n]
        o = nms_oracle.decode(x.cpu().numpy(), proto, z, W.alpha, W.alpha_ucn, W.beta, T, 2, 5)
        small = dec.decode(x, T=T, app=True, flags=True)
        assert np.array_equal(small.app.cpu().numpy(), o["app"])
        assert np.array_equal(small.flags.cpu().numpy(), flags[lo:lo + n])
    del llr
    torch.cuda.empty_cache()


@pytest.mark.parametrize("q", [4, 3])
def test_full_batch_q4_q3(cuda_device, q):
    """q = 4 / 3 at B = 2^20 on the bit-sliced kernel (grid step 1 / 2, qmax 7 / 3): counters and
    per-frame flags equal flood's, and the in-decoder channel gives the same."""
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    proto, g, W, cp = bench.load_problem(config="C2")
    dec = NMSDecoder(proto, 24, W, 2, q, device=cuda_device, B_max=B)
    assert dec.kernel_info()[1].startswith("bsl["), dec.kernel_info()
    sigma = float(cp.sigma(2.5))
    llr = dec.awgn(B, sigma, seed=37)
    res = {}
    for k in ("fused", "flood"):
        r = dec.decode(llr, app=False, counters=True, flags=True, kernel=k)
        res[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy())
    assert np.array_equal(res["fused"][0], res["flood"][0])
    assert np.array_equal(res["fused"][1], res["flood"][1])
    assert 0 < res["fused"][0][1] < B
    r = dec.decode_awgn(B, sigma, 37, counters=True, flags=True)
    assert np.array_equal(r.counters.cpu().numpy(), res["fused"][0])
    del llr
    torch.cuda.empty_cache()
