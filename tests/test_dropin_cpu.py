"""Drop-in contract on CPU: the Session facade + FER loop reproduce the reference's
``compute_results`` Results (fixture made by the reference itself).  The decoder behind the
Session here is the oracle (test infrastructure); the GPU version of this test is in
test_gpu_parity.py."""
import os
import sys

import numpy as np
import pytest

from conftest import GOLDEN, REFERENCE, ROOT
from _helpers import OracleDecoder
from ldpc_error_floor_amd import fer
from ldpc_error_floor_amd.code import TannerGraph, load_base_graph
from ldpc_error_floor_amd.session import Session, make_net_dict
from ldpc_error_floor_amd.weights import expand_weights


def _setup():
    d = np.load(os.path.join(GOLDEN, "results_wman_303.npz"))
    proto = load_base_graph(os.path.join(ROOT, "ldpc_error_floor_amd", "data", "BaseGraph",
                                         "wman_N0576_R34_z24.txt"))
    g = TannerGraph(proto, 24)
    W = expand_weights((3, 0, 3), {0: d["w0"], 2: d["w2"]}, 20, g)
    return d, proto, g, W


def test_session_shape_contract():
    d, proto, g, W = _setup()
    sess = Session(OracleDecoder(proto, 24, W), batch_size=4)
    nd = make_net_dict(20)
    X = np.full((4, 24, 24), -7.5)
    y, loss = sess.run([nd["ya_output_all"], nd["lossa"]],
                       {nd["xa"]: X, nd["ya"]: np.zeros((4, 576)), nd["etha"]: 0, nd["learn_rate"]: 0})
    assert y.shape == (80, 576) and y.dtype == np.float32 and loss == 0.0
    assert np.all(y < 0)          # noiseless all-zero word decodes
    with pytest.raises(ValueError):
        sess.run(nd["ya_output_all"], {nd["xa"]: X[:3]})


def test_fer_loop_reproduces_reference_results():
    d, proto, g, W = _setup()
    sess = Session(OracleDecoder(proto, 24, W), batch_size=int(d["B"]))
    wr, nr = np.random.RandomState(2044), np.random.RandomState(1076)
    Results, _ = fer.compute_results(int(d["sample_num"]), [], [], d["sigma"], wr, nr, int(d["B"]),
                                     0, g.N, g.M, 24, True, 20, sess, make_net_dict(20), 0, 2, 0, 0,
                                     0, 0, 5, 20.0)
    np.testing.assert_array_equal(Results, d["Results"])


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference not mounted")
def test_reference_compute_results_runs_on_session():
    """The reference's own, unmodified compute_results driving this package's Session."""
    d, proto, g, W = _setup()
    sys.path.insert(0, REFERENCE)
    try:
        import Print_Functions as PF
    finally:
        sys.path.remove(REFERENCE)
    sess = Session(OracleDecoder(proto, 24, W), batch_size=int(d["B"]))
    wr, nr = np.random.RandomState(2044), np.random.RandomState(1076)
    Results, _ = PF.compute_results(int(d["sample_num"]), [], [], d["sigma"], wr, nr, int(d["B"]),
                                    0, g.N, g.M, 24, True, 20, sess, make_net_dict(20), 0, 2, 0, 0,
                                    0, 0, 5, 20.0)
    np.testing.assert_array_equal(Results, d["Results"])
