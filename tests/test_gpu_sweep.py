"""fer_sweep / build_session / kernel selection details on the GPU: the decoder's puncture /
shorten ranges reach the sweep, an interrupted sweep resumes exactly, and a clip_LLR off the
quantizer grid makes AUTO choose the flood kernel instead of failing (GPU only)."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")
G5 = "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640"


def _g5_decoder(device, **kw):
    from ldpc_error_floor_amd.decoder import Decoder
    return Decoder(os.path.join(DATA, "BaseGraph", G5 + ".txt"), 64, punct=(1, 128),
                   short=(513, 640), sharing=(2, 2, 2),
                   weights_txt=os.path.join(DATA, "Results", "5G", G5 + "_Weight_End50.txt"),
                   T=20, device=device, **kw)


def _manual(dec, sigmas, n, seed, punct, short):
    import torch
    out = []
    for si, s in enumerate(sigmas):
        cnt = torch.zeros(4, dtype=torch.int64, device=dec.device)
        llr = dec.awgn(n, s, seed + 7919 * si, punct=punct, short=short)
        dec.decode(llr, app=False, counters=cnt)
        out.append(cnt.cpu().tolist())
    return out


def test_sweep_uses_decoder_puncture_and_shortening(cuda_device):
    from ldpc_error_floor_amd.code import CodeParams
    from ldpc_error_floor_amd.fer import fer_sweep
    dec = _g5_decoder(cuda_device)
    cp = CodeParams(dec.graph.proto, 64, 1, 128, 513, 640)
    sig = [float(cp.sigma(1.5)), float(cp.sigma(2.0))]
    res = fer_sweep(dec, sig, 3000, 1024, seed=21)
    got = [[r.bit_err_last, r.frame_err_last, r.frame_err_all, r.loss2] for r in res]
    assert got == _manual(dec, sig, 3000, 21, (1, 128), (513, 640))
    assert got != _manual(dec, sig, 3000, 21, (0, 0), (0, 0))
    # the collection path (awgn into HBM + decode) uses the same ranges
    res2 = fer_sweep(dec, sig[:1], 3000, 1024, seed=21, uncor_path=os.devnull)
    assert [res2[0].bit_err_last, res2[0].frame_err_last] == got[0][:2]


def test_build_session_carries_channel_ranges(cuda_device):
    from ldpc_error_floor_amd.config import NMSConfig
    from ldpc_error_floor_amd.session import build_session
    cfg = NMSConfig(filename=G5, sharing=(2, 2, 2), z_value=64, iters_max=20, batch_size=8,
                    punct_start=1, punct_end=128, short_start=513, short_end=640,
                    weights_file=os.path.join(DATA, "Results", "5G", G5 + "_Weight_End50.txt"))
    sess, _ = build_session(cfg, device=cuda_device)
    assert sess.decoder.punct == (1, 128) and sess.decoder.short == (513, 640)
    x = sess.decoder.awgn(4, 0.8, seed=1).cpu().numpy()
    assert np.all(x[:, :128] == 0) and np.all(x[:, 512:640] == -20)


def test_sweep_resume_on_gpu(cuda_device, tmp_path):
    from ldpc_error_floor_amd.fer import fer_sweep
    dec = _g5_decoder(cuda_device)
    sig = [0.85, 0.8]
    full = fer_sweep(dec, sig, 20000, 2048, seed=3)

    class Stop(Exception):
        pass

    n = {"c": 0}

    def progress(si, done, total):
        n["c"] += 1
        if n["c"] == 13:
            raise Stop()

    ck = str(tmp_path / "c.json")
    with pytest.raises(Stop):
        fer_sweep(dec, sig, 20000, 2048, seed=3, checkpoint=ck, checkpoint_every=3,
                  progress=progress)
    res = fer_sweep(dec, sig, 20000, 2048, seed=3, checkpoint=ck, resume=True)
    key = lambda rs: [(r.bit_err_last, r.frame_err_last, r.frame_err_all, r.loss2) for r in rs]  # noqa: E731
    assert key(res) == key(full)


@pytest.mark.parametrize("cfg", ["C2", "C5"])
def test_sweep_overlapped_channel_equals_inline(cuda_device, cfg):
    """fer_sweep's pipelined path (batch j + 1's channel kernel on a second stream while batch j
    decodes, for the kernels that read their LLRs from HBM: the float modes' ffl / flood) decodes
    exactly the codewords of the in-line path: several SNR points and a ragged last batch.  The
    QMS bit-sliced decodes generate their channel in the kernel's prologue and do not pipeline."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.fer import fer_sweep, _pipelines
    c = bench.CONFIGS[cfg]
    proto, g, W, cp = bench.load_problem(T=12, config=cfg)
    qms = NMSDecoder(proto, c["z"], W, 2, 5, device=cuda_device)
    assert qms.kernel_info()[1].startswith(("bsl[", "bsc[")) and not _pipelines(qms, None, None)
    dec = NMSDecoder(proto, c["z"], W, 1, 5, device=cuda_device)        # min-sum fp32
    dec.punct, dec.short = c.get("punct", (0, 0)), c.get("short", (0, 0))
    assert _pipelines(dec, None, None)
    sig = [float(cp.sigma(c["snr"] - 1.0)), float(cp.sigma(c["snr"] - 0.5))]
    key = lambda rs: [(r.bit_err_last, r.frame_err_last, r.frame_err_all, r.loss2) for r in rs]  # noqa: E731
    inline = key(fer_sweep(dec, sig, 9000, 2048, seed=4))
    assert key(fer_sweep(dec, sig, 9000, 2048, seed=4, overlap=True)) == inline
    assert inline[0][1] > 0


def test_off_grid_clip_selects_flood(cuda_device):
    """clip_LLR = 19.7 is not a multiple of the q=5 step: the fused kernel cannot clip in its
    integer domain, so AUTO must pick flood (and 'fused' is reported unsupported)."""
    import torch
    from ldpc_error_floor_amd.code import TannerGraph, load_base_graph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import flat_weights
    from oracle import nms_oracle
    proto = load_base_graph(os.path.join(DATA, "BaseGraph", "wman_N0576_R34_z24.txt"))
    W = flat_weights(TannerGraph(proto, 24), 10, 0.75)
    dec = NMSDecoder(proto, 24, W, 2, 5, clip_LLR=19.7, device=cuda_device)
    assert not dec.supports("fused") and dec.supports("flood")
    assert dec.kernel_info()[1] == "flood"
    llr = dec.awgn(64, 0.8, seed=2)
    app = dec.decode(llr, app=True).app.cpu().numpy()
    ref = nms_oracle.decode(llr.cpu().numpy(), proto, 24, W.alpha, W.alpha_ucn, W.beta, 10, 2,
                            5, clip=19.7)["app"]
    assert np.array_equal(app, ref)
    # the in-decoder channel falls back to generate-then-decode with the flood kernel
    got = dec.decode_awgn(64, 0.8, seed=2, app=True).app.cpu().numpy()
    assert np.array_equal(got, app)
    on_grid = NMSDecoder(proto, 24, W, 2, 5, clip_LLR=20.0, device=cuda_device)
    assert on_grid.supports("fused")
    torch.cuda.synchronize()
