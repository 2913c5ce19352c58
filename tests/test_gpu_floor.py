"""Error-floor events of the timed kernel (GPU only), and the C4 high-SNR flare at the end.  At
6 dB the wman decoder (C2: QMS q5, T=20, trained [3,0,3] weights) fails about 4e-7 of its frames (`profiles/r3/sweep_c2/`: 3,475
frames in 8.6e9 codewords).  The 2^20-codeword parity tests see none of these frames, so here
2^27 codewords at that SNR go through the bit-sliced kernel and through flood (both pinned on the
reference's fixtures) batch by batch: counters and per-frame flags must agree, there must be
failing frames, and the failing frames, decoded by the CPU oracle (the restatement of
`build_neural_network`, Main_Functions.py:157-335), must fail there too with the same APP."""
import numpy as np
import pytest

from oracle import nms_oracle

pytestmark = pytest.mark.gpu
B = 1 << 20
BATCHES = 128


def test_floor_events_bitsliced_equals_flood_and_oracle(cuda_device):
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = bench.CONFIGS["C2"]
    proto, g, W, cp = bench.load_problem(config="C2")
    T, z = cfg["T"], cfg["z"]
    dec = NMSDecoder(proto, z, W, 2, 5, device=cuda_device, B_max=B)
    assert dec.kernel_info(T)[1].startswith("bsl["), dec.kernel_info(T)
    sigma = float(cp.sigma(6.0))
    llr = torch.empty((B, dec.n_vars), dtype=torch.float32, device=cuda_device)
    tot = {k: np.zeros(4, np.int64) for k in ("fused", "flood")}
    fails = []                                    # (batch, frame) of the bit-sliced kernel's failures
    for b in range(BATCHES):
        dec.awgn(B, sigma, seed=4242, offset=b * B, out=llr)
        flags = {}
        for k in ("fused", "flood"):
            r = dec.decode(llr, T=T, app=False, counters=True, flags=True, kernel=k)
            tot[k] += r.counters.cpu().numpy()
            flags[k] = r.flags.cpu().numpy()
        assert dec.last_kernel() == "flood"
        assert np.array_equal(flags["fused"], flags["flood"]), b
        for f in np.nonzero((flags["fused"] >> 1) & 1)[0][:2]:
            if len(fails) < 6:
                fails.append((b, int(f), llr[int(f)].cpu().numpy().copy()))
    assert np.array_equal(tot["fused"], tot["flood"]), (tot["fused"], tot["flood"])
    n = BATCHES * B
    assert 0 < tot["fused"][1] < 1e-5 * n, tot["fused"]           # a floor event rate, not a waterfall
    # the failing frames against the oracle: they fail there too, with the same APP at every t
    x = np.stack([v for _, _, v in fails])
    o = nms_oracle.decode(x, proto, z, W.alpha, W.alpha_ucn, W.beta, T, 2, 5)
    r = dec.decode(torch.from_numpy(x).to(cuda_device), T=T, app=True, flags=True)
    assert np.array_equal(r.app.cpu().numpy(), o["app"])
    assert np.all((r.flags.cpu().numpy() >> 1) & 1 == 1)
    assert np.all(o["hard"][T - 1].reshape(len(fails), -1).any(axis=1))
    del llr
    torch.cuda.empty_cache()


def test_bg2_high_snr_flare_bitsliced_equals_flood_and_oracle(cuda_device):
    """5G BG2 (C4: trained [2,2,2] weights with UCN, puncture 1-128, shorten 513-640): above
    2.5 dB its FER rises again (`profiles/r3/sweep_c4/`), with single wrong bits in the degree-1
    extension columns.  At 4 dB the bit-sliced kernel equals flood frame by frame and the oracle
    decodes the failing frames to the same APP at every iteration."""
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    cfg = bench.CONFIGS["C4"]
    proto, g, W, cp = bench.load_problem(config="C4")
    T, z = cfg["T"], cfg["z"]
    dec = NMSDecoder(proto, z, W, 2, 5, device=cuda_device, B_max=B)
    dec.punct, dec.short = cfg["punct"], cfg["short"]
    llr = dec.awgn(B, float(cp.sigma(4.0)), seed=99)
    res = {}
    for k in ("fused", "flood"):
        r = dec.decode(llr, T=T, app=False, counters=True, flags=True, kernel=k)
        res[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy(), dec.last_kernel())
    assert res["fused"][2].startswith("bsl[") and res["flood"][2] == "flood"
    assert np.array_equal(res["fused"][0], res["flood"][0])
    assert np.array_equal(res["fused"][1], res["flood"][1])
    fail = np.nonzero((res["fused"][1] >> 1) & 1)[0]
    assert 1e-3 * B < len(fail) < 0.1 * B
    x = llr[torch.from_numpy(fail[:8]).to(cuda_device)].cpu().numpy()
    o = nms_oracle.decode(x, proto, z, W.alpha, W.alpha_ucn, W.beta, T, 2, 5)
    small = dec.decode(torch.from_numpy(x).to(cuda_device), T=T, app=True, flags=True)
    assert np.array_equal(small.app.cpu().numpy(), o["app"])
    assert np.all(o["hard"][T - 1].reshape(len(x), -1).any(axis=1))
    del llr
    torch.cuda.empty_cache()
