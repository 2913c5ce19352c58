"""The boosting pipeline's post-decoder path end to end on the GPU (SURVEY §8 f rank 2):
regenerate the stripped Inputs/[Uncor]_* files with the base decoder (sampling_type 2 as a GPU
sweep), read them back with process_data's restatement, and evaluate the post decoder over
them with compute_results(sampling_type=1) through the Session facade; then the host-side
sampling_type=2 collection through the Session.  Every Results array and file must equal the
ones the oracle-backed Session produces (Main_Functions.py:526-576, Print_Functions.py:6-10,
:120-126, :130-165)."""
import os

import numpy as np
import pytest

from conftest import ROOT, load_case
from _helpers import OracleDecoder, flags_from_app
from oracle import nms_oracle

pytestmark = pytest.mark.gpu
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")
NAME = "wman_N0576_R34_z24"


def _base(device):
    from ldpc_error_floor_amd.decoder import Decoder
    return Decoder(os.path.join(DATA, "BaseGraph", NAME + ".txt"), 24, sharing=(3, 0, 3),
                   weights_txt=os.path.join(DATA, "Weights", f"C0_{NAME}_Opt_Weight_End20.txt"),
                   T=20, device=device)


def test_uncor_inputs_then_post_decoder_results(cuda_device, tmp_path):
    from ldpc_error_floor_amd import fer
    from ldpc_error_floor_amd.channel import load_uncor_inputs
    from ldpc_error_floor_amd.code import CodeParams
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.session import Session, make_net_dict
    base = _base(cuda_device)
    sigma = float(CodeParams(base.graph.proto, 24).sigma(2.5))
    res = fer.collect_uncor_inputs(base, sigma, NAME, (200, 60, 60), str(tmp_path), batch=4096,
                                   seed=17)
    assert sorted(r for r, _ in res.values()) == [60, 60, 200]
    tr, trc, va, vac, te, tec = load_uncor_inputs(NAME, 200, 1, 60, 1, 60, str(tmp_path))
    # every collected word is one the base decoder fails at every iteration (oracle check)
    W = base.weights
    o = nms_oracle.decode(-tr[:40], base.graph.proto, 24, W.alpha, W.alpha_ucn, W.beta, 20, 2, 5)
    assert np.all(flags_from_app(o["app"]) & 1)
    # post decoder: the 30-iteration base+post cascade ([3,3,3]) over the uncorrected words
    c = load_case("wman_333_post_snr2.0")
    B = 20
    gpu = Session(NMSDecoder(c["g"].proto, 24, c["W"], 2, 5, device=cuda_device), B)
    cpu = Session(OracleDecoder(c["g"].proto, 24, c["W"]), B)
    nd = make_net_dict(30)
    for llr, cw, n in ((tr, trc, 200), (va, vac, 60), (te, tec, 60)):
        args = (n, llr, cw, np.array([0.0]), None, None, B, 1, 24, 6, 24, True, 30)
        tail = (nd, 0, 2, 0, 0, 0, 0, 5, 20.0)
        r_gpu, _ = fer.compute_results(*args, gpu, *tail)
        r_cpu, _ = fer.compute_results(*args, cpu, *tail)
        np.testing.assert_array_equal(r_gpu, r_cpu)
        assert r_gpu[2, 0] < 1.0      # the post iterations correct some of them


def test_session_sampling_type2_collection(cuda_device, tmp_path):
    from ldpc_error_floor_amd import fer
    from ldpc_error_floor_amd.code import CodeParams
    from ldpc_error_floor_amd.session import Session, make_net_dict
    base = _base(cuda_device)
    sigma = np.array([float(CodeParams(base.graph.proto, 24).sigma(2.0))])
    out = {}
    for tag, dec in (("gpu", base), ("cpu", OracleDecoder(base.graph.proto, 24, base.weights))):
        path = str(tmp_path / f"Uncor_{tag}.txt")
        wr, nr = np.random.RandomState(2044), np.random.RandomState(1076)
        R, _ = fer.compute_results(120, [], [], sigma, wr, nr, 40, 2, 24, 6, 24, True, 20,
                                   Session(dec, 40), make_net_dict(20), 0, 2, 0, 0, 0, 0, 5, 20.0,
                                   uncor_path=path)
        out[tag] = (R, open(path).read())
    np.testing.assert_array_equal(out["gpu"][0], out["cpu"][0])
    assert out["gpu"][1] == out["cpu"][1] and out["gpu"][1].count("\n") > 10
