"""The CPU oracle against the golden fixtures generated from the reference (CPU only)."""
import numpy as np
import pytest

from conftest import DECODER_CASES, load_case
from oracle import nms_oracle

MS_ATOL = 1e-3   # SURVEY.md §8 c: fp32 summation-order tolerance for MS soft values


@pytest.mark.parametrize("name", DECODER_CASES)
def test_oracle_matches_reference(name):
    c = load_case(name)
    W = c["W"]
    out = nms_oracle.decode(c["llr"], c["g"].proto, c["z"], W.alpha, W.alpha_ucn, W.beta, c["T"],
                            c["dt"], c["q"])
    app = out["app"][:, :, :c["Nt"] * c["z"]]
    if c["exact"]:
        assert np.array_equal(app, c["app"]), "QMS soft output must be bit-exact"
    else:
        np.testing.assert_allclose(app, c["app"], rtol=0, atol=MS_ATOL)
    assert np.array_equal(out["hard"], c["hard"])
    assert np.array_equal(out["synd"], c["synd"])


def test_fixture_inventory():
    # the SURVEY §8 c list: wman base, post cascade, MS, all q_bits, 802.11n, 5G BG2, z=1
    need = {"wman_303_q5_snr2.0", "wman_303_q5_snr2.5", "wman_303_q5_snr3.5",
            "wman_333_post_snr2.0", "wman_303_sp_snr2.5", "wman_333_sp_snr2.0",
            "g5bg2_222_sp_snr2.0",
            "wman_303_ms_snr2.5", "wman_222_q6", "wman_222_qm5", "wman_222_q4", "wman_222_q3",
            "wifi_333_q5_snr3.0", "g5bg2_222_q5_snr2.0", "mackay_333_q5_snr2.5",
            "polar_222_q5_snr3.0", "g5bg1_303_flat_t50_snr2.5"}
    assert need <= set(DECODER_CASES)


def test_quantizer_grid():
    x = np.array([-100, -7.74, -7.75, -0.25, -0.24, 0, 0.25, 0.26, 0.75, 1.25, 7.6, 100], np.float32)
    np.testing.assert_array_equal(nms_oracle.quantize(x, 5),
                                  [-7.5, -7.5, -7.5, -0.0, -0.0, 0, 0, 0.5, 1.0, 1.0, 7.5, 7.5])
    np.testing.assert_array_equal(nms_oracle.quantize(np.float32([15.7, 2.5, 3.5]), 6), [15.5, 2, 4])
    np.testing.assert_array_equal(nms_oracle.quantize(np.float32([3.0, 5.0, -9]), 3), [4, 4, -6])


@pytest.mark.parametrize("name", ["wman_303_q5_snr2.0", "wman_333_post_snr2.0", "wman_111_q5",
                                  "wifi_333_q5_snr3.0", "polar_222_q5_snr3.0", "wman_303_ms_snr2.5"])
def test_dense_baseline_matches_reference(name):
    """The dense TF-graph-equivalent CPU baseline computes the same decoder."""
    from oracle import nms_dense
    c = load_case(name)
    W = c["W"]
    out = nms_dense.decode(c["llr"], c["g"].proto, c["z"], W.alpha, W.alpha_ucn, W.beta, c["T"],
                           c["dt"], c["q"])
    app = out["app"][:, :, :c["Nt"] * c["z"]]
    if c["exact"]:
        assert np.array_equal(app, c["app"])
    else:
        np.testing.assert_allclose(app, c["app"], rtol=0, atol=MS_ATOL)
