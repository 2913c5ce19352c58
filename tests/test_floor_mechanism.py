"""The C4 (5G BG2 n1024, [2,2,2] trained weights, q5, T=20) FER "flare" is the channel
saturation of its degree-1 bits, not a decoder defect (CPU only, from the committed sweep).

Mechanism.  BG2's columns 14-19 have degree 1: 6 x 64 = 384 bits, each with one check.  At the
last iteration the check's message to such a bit has magnitude Q(relu(alpha_19 m)) with m <= 7.5
(V->C clamped by the q5 quantizer, Main_Functions.py:227) and the trained alpha_19 = 0.988 of
those rows, so at most Q(7.41) = 7.5.  The APP adds the unweighted quantized channel LLR
(Main_Functions.py:317-325): a bit whose channel LLR rounds to +7.5 (raw LLR >= 7.25) ends at
APP >= 7.5 - 7.5 = 0, and the reference's hard decision is APP >= 0 (calc_ber_fer,
Print_Functions.py:100-118): a 1, i.e. a frame error at the last iteration, whatever the other
bits do.  P(raw LLR >= 7.25) = Q(7.25 sigma / 2 + 1 / sigma) for LLR = 2 (sigma n - 1) / sigma^2
(create_mix_epoch, :29-72), and 7.25 sigma / 2 + 1 / sigma *falls* as sigma falls while
sigma > sqrt(2 / 7.25) = 0.525 (below 5.6 dB here), so this floor rises with SNR.
FER_pred = 1 - (1 - Q(.))^384 reproduces the measured FER_last of the 2^24-codeword sweep
(profiles/r3/sweep_c4/sweep_c4.json) to within 1.1 % at 3.0-4.0 dB, where 98-99 % of the failed
frames have a single wrong bit."""
import json
import os

import numpy as np

from conftest import ROOT


def _q5(x):
    return float(np.clip(np.round(np.float32(x) * 2) / 2, -7.5, 7.5))


def test_c4_flare_is_degree1_saturation():
    import sys
    from scipy.special import ndtr
    sys.path.insert(0, ROOT)
    import bench
    proto, g, W, cp = bench.load_problem(config="C4")
    P = np.asarray(proto)
    deg = (P >= 0).sum(axis=0)
    cols = np.flatnonzero(deg == 1)
    assert cols.tolist() == [14, 15, 16, 17, 18, 19]
    edges = [(i, j) for i in range(P.shape[0]) for j in range(P.shape[1]) if P[i, j] >= 0]
    T = W.T
    for j in cols:
        e = next(k for k, (_, jj) in enumerate(edges) if jj == j)
        # the strongest message the check can send at the last iteration (SCN and UCN weight)
        m = max(_q5(np.float32(W.alpha[T - 1, e]) * np.float32(7.5)),
                _q5(np.float32(W.alpha_ucn[T - 1, e]) * np.float32(7.5)))
        assert m == 7.5                 # ties a saturated +7.5 channel LLR at APP = 0 -> bit 1
    n_bits = len(cols) * 64
    with open(os.path.join(ROOT, "profiles", "r3", "sweep_c4", "sweep_c4.json")) as f:
        sweep = json.load(f)
    for r in sweep["scan"]:
        s = r["sigma"]
        p_bit = ndtr(-(7.25 * s / 2 + 1 / s))
        pred = 1.0 - (1.0 - p_bit) ** n_bits
        if r["snr_db"] >= 3.0:
            assert abs(pred / r["fer_last"] - 1) < 0.011, (r["snr_db"], pred, r["fer_last"])
            # failed frames carry about one wrong bit: the saturated degree-1 bit
            assert r["bit_err_last"] / r["frame_err_last"] < 1.05
        elif r["snr_db"] >= 2.5:
            assert 0.9 < r["fer_last"] / pred < 1.1
    # the rise with SNR: the argument 7.25 s / 2 + 1 / s decreases while s > sqrt(2 / 7.25)
    sig = [r["sigma"] for r in sweep["scan"] if r["snr_db"] >= 2.5]
    assert all(x > np.sqrt(2 / 7.25) for x in sig)
    fers = [r["fer_last"] for r in sweep["scan"] if r["snr_db"] >= 2.5]
    assert fers == sorted(fers)


def test_c5_floor_is_degree1_saturation_over_ten_decades():
    """The same mechanism with C5's flat weights (5G BG1 n2112, alpha = 0.75, beta = 1, q5,
    T = 50): BG1's 432 degree-1 bits (columns 26-31) get at most Q(0.75 x 7.5) = 5.5 from their
    check, so a channel LLR that rounds to >= 5.5 (raw >= 5.25) leaves APP >= 0, a frame error.
    FER = 1 - (1 - Q(5.25 sigma / 2 + 1 / sigma))^432 predicts every committed C5 sweep point
    (profiles/r2/sweep_c5*, profiles/r5/sweep_c5: 4.2e6 to 1.7e10 codewords per point, 3 to 15
    dB, FER 0.22 down to 1.7e-10) within Poisson noise."""
    import sys
    from scipy.special import ndtr
    sys.path.insert(0, ROOT)
    import bench
    proto, g, W, cp = bench.load_problem(config="C5")
    P = np.asarray(proto)
    cols = np.flatnonzero((P >= 0).sum(axis=0) == 1)
    assert cols.tolist() == list(range(26, 32))
    assert np.all(W.alpha == np.float32(0.75)) and np.all(W.beta == np.float32(1.0))
    assert _q5(np.float32(0.75) * np.float32(7.5)) == 5.5
    n_bits = len(cols) * 72
    pts = []
    for f in ("r2/sweep_c5/sweep_c5.json", "r2/sweep_c5_deep/sweep_c5_14.5dB.json",
              "r2/sweep_c5_deep/sweep_c5_15dB.json",
              "r5/sweep_c5/sweep_c5.json"):       # (round 5: 1.7e10 codewords at 15 dB, 3 frames)
        with open(os.path.join(ROOT, "profiles", f)) as fh:
            d = json.load(fh)
        pts += d.get("scan", []) + d["deep"]
    assert len(pts) >= 16
    for r in pts:
        s, n = r["sigma"], r["codewords"]
        p_bit = ndtr(-(5.25 * s / 2 + 1 / s))
        exp = n * (1.0 - (1.0 - p_bit) ** n_bits)
        obs = r["frame_err_last"]
        # Poisson noise, plus 0.5 % for the frames the mechanism does not cover at low SNR
        assert abs(obs - exp) <= 4.0 * np.sqrt(exp) + 0.005 * exp + 3, (r["snr_db"], obs, exp)
