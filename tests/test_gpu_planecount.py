"""The bit-sliced kernels' variable phase runs at the fewest planes of S each place's largest
degree allows (ldpc_bs_kernel.h BS_SBV, ldpc_bsc.hip BSC_SBV: 7 planes where 15 dw + 15 <= 63, 8
where <= 127, else 9), and 802.11n keeps every C->V of its degree-4 variables in registers
(BS_KEEP_DV).  These bounds are tight exactly when every message is saturated, so the decodes
here drive them there: channel LLRs at the largest grid magnitude (a very high SNR) with a share
of their signs flipped, and the trained / flat weights scaled up so that Q(beta ch) and
Q(alpha m) saturate too.  Counters, frame flags and per-iteration frame-error words must equal
the flood kernel's, which the reference fixtures pin (GPU only)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _saturated_llr(dec, cp, B, flip, seed):
    """LLRs at the grid's largest magnitude, a share `flip` of them negated (punctured and
    shortened positions keep their values)"""
    import torch
    llr = dec.awgn(B, float(cp.sigma(40.0)), seed=seed)          # every level at the grid's end
    rng = np.random.RandomState(seed)
    f = rng.uniform(size=tuple(llr.shape)) < flip
    for lo, hi in (dec.punct, dec.short):                         # 1-based inclusive ranges
        if lo > 0:
            f[:, lo - 1:hi] = False
    sign = np.where(f, -1.0, 1.0).astype(np.float32)
    return llr * torch.from_numpy(sign).to(llr.device)


@pytest.mark.parametrize("cfg", ["C2", "C3", "C4", "C5"])
@pytest.mark.parametrize("flip", [0.0, 0.02, 0.3])
def test_saturated_messages_equal_flood(cuda_device, cfg, flip):
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    c = bench.CONFIGS[cfg]
    T = 8
    proto, g, W, cp = bench.load_problem(T=T, config=cfg)
    W.alpha = (np.asarray(W.alpha) * 1.6).astype(np.float32)
    W.beta = (np.asarray(W.beta) * 2.0).astype(np.float32)
    if W.alpha_ucn is not None:
        W.alpha_ucn = (np.asarray(W.alpha_ucn) * 1.6).astype(np.float32)
    dec = NMSDecoder(proto, c["z"], W, 2, 5, device=cuda_device)
    dec.punct, dec.short = c.get("punct", (0, 0)), c.get("short", (0, 0))
    assert dec.kernel_info()[1].startswith(("bsl[", "bsc[")), dec.kernel_info()
    llr = _saturated_llr(dec, cp, 3001, flip, 11)
    out, iw = {}, {}
    for k in ("flood", "fused"):
        r = dec.decode(llr, app=False, counters=True, flags=True, kernel=k, iter_wrong=True)
        out[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy())
        iw[k] = r.iter_wrong.cpu().numpy()
        if k == "fused":
            assert dec.last_kernel().startswith(("bsl[", "bsc[")), dec.last_kernel()
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    assert np.array_equal(iw["fused"], iw["flood"])
