"""The uncorrected-word sweep on the in-kernel channel (GPU only).

``fer_sweep(uncor_path=...)`` decodes with ``ldpc_decode_awgn`` (the channel generated inside
the decoder) and regenerates only the failing frames' LLR rows (``ldpc_channel_awgn_rows``).
Those rows must be the rows ``ldpc_channel_awgn`` writes, bit for bit, so the file is the one
the HBM-channel path (``awgn`` + ``decode`` + ``collect_uncorrected``, the reference's
``compute_results`` -> ``write_uncor_file``, ``Print_Functions.py:120-126``) writes."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")


def _decoder(case, device):
    from ldpc_error_floor_amd.code import CodeParams, TannerGraph, load_base_graph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights, read_weight_file
    if case.startswith("wman"):
        proto = load_base_graph(os.path.join(DATA, "BaseGraph", "wman_N0576_R34_z24.txt"))
        g = TannerGraph(proto, 24)
        wf = read_weight_file(os.path.join(DATA, "Weights", "C0_wman_N0576_R34_z24_Opt_Weight_End20.txt"))
        W = expand_weights((3, 0, 3), {0: wf.blocks[0], 2: wf.blocks[2]}, 20, g)
        dt = 0 if case == "wman_sp" else 2
        return NMSDecoder(proto, 24, W, dt, 5, device=device), CodeParams(proto, 24), (0, 0), (0, 0)
    name = "5G_LDPC_R0.50_n_dec1280_n1024_k512_z64_s513_640"
    proto = load_base_graph(os.path.join(DATA, "BaseGraph", name + ".txt"))
    g = TannerGraph(proto, 64)
    wf = read_weight_file(os.path.join(DATA, "Results", "5G", name + "_Weight_End50.txt"))
    W = expand_weights((2, 2, 2), wf.blocks, 20, g)
    dec = NMSDecoder(proto, 64, W, 2, 5, device=device)
    return dec, CodeParams(proto, 64, 1, 128, 513, 640), (1, 128), (513, 640)


@pytest.mark.parametrize("case", ["wman_qms", "bg2_qms", "wman_sp"])
def test_channel_rows_equal_channel(cuda_device, case):
    """ldpc_channel_awgn_rows == the rows of ldpc_channel_awgn at any index list (unaligned
    offset, unsorted indices, repeats), QMS level sampler and float Box-Muller alike."""
    import torch
    dec, cp, punct, short = _decoder(case, cuda_device)
    B, off, seed = 1000 + 13, 4096 + 3, 77
    sigma = float(cp.sigma(2.0))
    llr = dec.awgn(B, sigma, seed, offset=off, punct=punct, short=short)
    rng = np.random.default_rng(5)
    idx_h = np.concatenate([rng.integers(0, B, 200), [0, B - 1, B - 1, 1, 2, 3]]).astype(np.int64)
    idx = torch.from_numpy(idx_h).to(cuda_device)
    rows = torch.empty((idx_h.size, dec.n_vars), dtype=torch.float32, device=cuda_device)
    dec._ext.channel_awgn_rows(rows.data_ptr(), idx.data_ptr(), idx_h.size, dec.n_vars, sigma, seed,
                               off, dec.decoding_type, dec.q_bit, punct[0], punct[1], short[0],
                               short[1], dec.clip, torch.cuda.current_stream(cuda_device).cuda_stream)
    torch.cuda.synchronize(cuda_device)
    assert torch.equal(rows, llr[idx])


@pytest.mark.parametrize("case", ["wman_qms", "bg2_qms"])
def test_collect_after_decode_awgn(cuda_device, case):
    """decode_awgn's frame flags equal decode's; the rows collect_uncorrected_awgn regenerates
    equal the HBM channel's rows of the same frames."""
    dec, cp, punct, short = _decoder(case, cuda_device)
    B, off, seed = 3001, 8 * 1024 + 1, 11
    sigma = float(cp.sigma(1.5 if case == "wman_qms" else 1.0))
    llr = dec.awgn(B, sigma, seed, offset=off, punct=punct, short=short)
    ref = dec.decode(llr, app=False, flags=True)
    got = dec.decode_awgn(B, sigma, seed, offset=off, punct=punct, short=short, flags=True)
    assert np.array_equal(got.flags.cpu().numpy(), ref.flags.cpu().numpy())
    a = dec.collect_uncorrected(ref.flags, llr)
    b = dec.collect_uncorrected_awgn(got.flags, sigma, seed, offset=off, punct=punct, short=short)
    assert a.shape[0] > 0 and np.array_equal(a, b)


def test_sweep_file_equals_hbm_channel_file(cuda_device, tmp_path):
    """fer_sweep(uncor_path=...) on the in-kernel channel writes the file the HBM-channel path
    writes, byte for byte (two SNR points, ragged last batch)."""
    from ldpc_error_floor_amd.channel import append_uncor_rows
    from ldpc_error_floor_amd.fer import fer_sweep
    dec, cp, punct, short = _decoder("wman_qms", cuda_device)
    sigmas = [float(cp.sigma(1.5)), float(cp.sigma(2.0))]
    n, batch, seed = 5000, 2048, 3
    path = tmp_path / "Uncor.txt"
    res = fer_sweep(dec, sigmas, n, batch, seed=seed, uncor_path=str(path))
    exp = tmp_path / "expected.txt"
    for si, sg in enumerate(sigmas):
        ps = seed + 7919 * si                      # fer_sweep's default point seeds
        for pos in range(0, n, batch):
            b = min(batch, n - pos)
            llr = dec.awgn(b, sg, ps, offset=pos)
            r = dec.decode(llr, app=False, flags=True)
            rows = dec.collect_uncorrected(r.flags, llr)
            if rows.shape[0]:
                append_uncor_rows(rows, str(exp), formatter=dec.format_uncor_rows)
    assert path.read_bytes() == exp.read_bytes()
    assert sum(x.frame_err_all for x in res) == path.read_bytes().count(b"\n") > 0


def test_sweep_checkpointed_and_resumed_file(cuda_device, tmp_path):
    """With a checkpoint after every batch (the deferred collection flushed before each save) and
    a resume of the finished sweep, the file and the counters equal the uninterrupted run's."""
    from ldpc_error_floor_amd.fer import fer_sweep
    dec, cp, punct, short = _decoder("wman_qms", cuda_device)
    sigmas = [float(cp.sigma(1.5))]
    a, b = tmp_path / "a.txt", tmp_path / "b.txt"
    ra = fer_sweep(dec, sigmas, 4500, 1024, seed=9, uncor_path=str(a))
    rb = fer_sweep(dec, sigmas, 4500, 1024, seed=9, uncor_path=str(b),
                   checkpoint=str(tmp_path / "ck.json"), checkpoint_every=1)
    assert a.read_bytes() == b.read_bytes() and a.stat().st_size > 0
    rc = fer_sweep(dec, sigmas, 4500, 1024, seed=9, uncor_path=str(b),
                   checkpoint=str(tmp_path / "ck.json"), checkpoint_every=1, resume=True)
    assert a.read_bytes() == b.read_bytes()
    assert [x.frame_err_all for x in ra] == [x.frame_err_all for x in rb] == [x.frame_err_all for x in rc]


@pytest.mark.parametrize("q_bit", [6, -5, 4, 3])
def test_channel_rows_every_quantizer(cuda_device, q_bit):
    """The rows of the index list on every QMS grid (the level sampler's thresholds differ per
    q_bit), MS fp32 included (q = 5 decoder, decoding type 1)."""
    import torch
    from ldpc_error_floor_amd.decoder import NMSDecoder
    dec0, cp, punct, short = _decoder("wman_qms", cuda_device)
    for dt, q in ((2, q_bit), (1, 5)):
        dec = NMSDecoder(dec0.graph.proto, 24, dec0.weights, dt, q, device=cuda_device)
        B, off, seed = 777, 12345, 5
        sigma = float(cp.sigma(1.0))
        llr = dec.awgn(B, sigma, seed, offset=off)
        idx_h = np.arange(B - 1, -1, -7, dtype=np.int64)
        idx = torch.from_numpy(idx_h).to(cuda_device)
        rows = torch.empty((idx_h.size, dec.n_vars), dtype=torch.float32, device=cuda_device)
        dec._ext.channel_awgn_rows(rows.data_ptr(), idx.data_ptr(), idx_h.size, dec.n_vars, sigma,
                                   seed, off, dec.decoding_type, dec.q_bit, 0, 0, 0, 0, dec.clip,
                                   torch.cuda.current_stream(cuda_device).cuda_stream)
        torch.cuda.synchronize(cuda_device)
        assert torch.equal(rows, llr[idx]), (dt, q)
