"""Error-floor events of the timed kernel (GPU only).  At 6 dB the wman decoder (C2: QMS q5,
T=20, trained [3,0,3] weights) fails about 4e-7 of its frames (`profiles/r3/sweep_c2/`: 3,475
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
