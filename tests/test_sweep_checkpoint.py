"""fer_sweep checkpoint / resume (per-SNR counters saved periodically for
multi-hour 1e-9 sweeps) on CPU with the oracle-backed stand-in decoder: an interrupted sweep
resumed from its checkpoint returns exactly the counters (and uncorrected-word file) of an
uninterrupted one."""
import json
import os

import numpy as np
import pytest

from test_distributed import SIGMAS, _make_decoder
from ldpc_error_floor_amd.fer import fer_sweep

N_CW, BATCH = 45, 8


class Stop(Exception):
    pass


def _tuples(res):
    return [(c.bit_err_last, c.frame_err_last, c.frame_err_all, c.loss2) for c in res]


def _interrupt_after(n):
    calls = {"n": 0}

    def progress(si, done, total):
        calls["n"] += 1
        if calls["n"] == n:
            raise Stop()
    return progress


@pytest.mark.parametrize("stop_at", [3, 7, 12])
def test_resume_equals_uninterrupted(tmp_path, stop_at):
    dec = _make_decoder()
    full = _tuples(fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076))
    ck = str(tmp_path / "sweep.ckpt")
    with pytest.raises(Stop):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, checkpoint=ck, checkpoint_every=2,
                  progress=_interrupt_after(stop_at))
    st = json.load(open(ck))
    assert st["done"] is False and (st["si"], st["pos"]) != (0, 0)
    res = fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, checkpoint=ck, checkpoint_every=2,
                    resume=True)
    assert _tuples(res) == full
    assert json.load(open(ck))["done"] is True
    # resuming a finished sweep decodes nothing and returns the same totals
    again = fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, checkpoint=ck, resume=True,
                      progress=_interrupt_after(1))
    assert _tuples(again) == full


def test_resume_uncorrected_file_not_duplicated(tmp_path):
    dec = _make_decoder()
    ref_path = str(tmp_path / "ref.txt")
    full = _tuples(fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=ref_path))
    path, ck = str(tmp_path / "Uncor.txt"), str(tmp_path / "u.ckpt")
    with pytest.raises(Stop):
        fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=path, checkpoint=ck,
                  checkpoint_every=2, progress=_interrupt_after(5))
    res = fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=path, checkpoint=ck,
                    checkpoint_every=2, resume=True)
    assert _tuples(res) == full and full[0][2] > 0
    assert open(path).read() == open(ref_path).read()


def test_resume_refuses_a_different_sweep(tmp_path):
    dec = _make_decoder()
    ck = str(tmp_path / "s.ckpt")
    with pytest.raises(Stop):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, checkpoint=ck, checkpoint_every=1,
                  progress=_interrupt_after(2))
    with pytest.raises(ValueError, match="checkpoint is for"):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1077, checkpoint=ck, resume=True)
    # without resume the checkpoint is overwritten from the start
    res = fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1077, checkpoint=ck)
    assert json.load(open(ck))["key"]["seed"] == 1077 and len(res) == 2


def test_collect_uncor_inputs_roundtrip(tmp_path):
    """collect_uncor_inputs writes the three post-decoder input files in the reference's row
    format; process_data's restatement reads them back, and every row is a frame the base
    decoder gets wrong at every iteration."""
    from _helpers import flags_from_app
    from ldpc_error_floor_amd.channel import load_uncor_inputs
    from ldpc_error_floor_amd.fer import collect_uncor_inputs
    from oracle import nms_oracle
    dec = _make_decoder()
    res = collect_uncor_inputs(dec, 0.7943282, "wman_N0576_R34_z24", (5, 3, 2), str(tmp_path),
                               batch=16, seed=9)
    assert sorted(v[0] for v in res.values()) == [2, 3, 5]
    tr, trc, va, vac, te, tec = load_uncor_inputs("wman_N0576_R34_z24", 5, 1, 3, 1, 2,
                                                  inputs_dir=str(tmp_path))
    assert tr.shape == (5, 576) and va.shape == (3, 576) and te.shape == (2, 576)
    assert not trc.any()
    x = -np.concatenate([tr, va, te])             # files hold negated LLRs
    o = nms_oracle.decode(x, dec.proto, 24, dec.W.alpha, dec.W.alpha_ucn, dec.W.beta, 20, 2, 5)
    assert np.all(flags_from_app(o["app"]) & 1)


def test_resume_refuses_a_different_decoder(tmp_path):
    """The checkpoint key carries the decoder (graph + weights hash, z, mode, q, clip, T): a
    resume with other weights or another iteration count is refused instead of adding the old
    counters to the new run."""
    from ldpc_error_floor_amd.weights import flat_weights
    from ldpc_error_floor_amd.code import TannerGraph
    dec = _make_decoder()
    ck = str(tmp_path / "d.ckpt")
    with pytest.raises(Stop):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=3, checkpoint=ck, checkpoint_every=1,
                  progress=_interrupt_after(2))
    other = _make_decoder()
    other.W = flat_weights(TannerGraph(other.proto, 24), 20, alpha=0.7, beta=1.0)
    with pytest.raises(ValueError, match="checkpoint is for"):
        fer_sweep(other, SIGMAS, N_CW, BATCH, seed=3, checkpoint=ck, resume=True)
    with pytest.raises(ValueError, match="checkpoint is for"):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=3, T=12, checkpoint=ck, resume=True)
    # the same decoder resumes
    full = _tuples(fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=3))
    assert _tuples(fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=3, checkpoint=ck, resume=True)) == full


def test_fresh_start_keeps_earlier_rows_and_resume_drops_its_own(tmp_path):
    """A checkpointed sweep appends to its uncorrected-word file like the reference
    (Print_Functions.py:122) and like an un-checkpointed sweep: rows earlier sweeps wrote stay.
    Its fresh start records the file's length in the checkpoint at once, so an attempt that
    dies before its first periodic checkpoint and is resumed leaves no duplicated rows."""
    dec = _make_decoder()
    ref_path = str(tmp_path / "ref.txt")
    fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=ref_path)
    ref = open(ref_path).read()
    assert ref
    prior = "0.0\t0.0\t0.0\trow of an earlier SNR point's sweep\n"
    path = tmp_path / "Uncor.txt"
    path.write_text(prior)
    fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=str(path),
              checkpoint=str(tmp_path / "a.ckpt"))
    assert path.read_text() == prior + ref
    # dies after 4 of 6 batches, before any periodic checkpoint (every 64 batches)
    path.write_text(prior)
    ck = str(tmp_path / "b.ckpt")
    with pytest.raises(Stop):
        fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=str(path), checkpoint=ck,
                  progress=_interrupt_after(4))
    st = json.load(open(ck))
    assert (st["si"], st["pos"], st["uncor_bytes"]) == (0, 0, len(prior))
    fer_sweep(dec, SIGMAS[:1], N_CW, BATCH, seed=5, uncor_path=str(path), checkpoint=ck,
              resume=True)
    assert path.read_text() == prior + ref


def test_resume_refuses_another_channel_stream(tmp_path, monkeypatch):
    """A checkpoint written under another on-GPU channel stream (fer.CHANNEL_STREAM: e.g. a
    round-3 file from the Box-Muller QMS channel) is refused, not resumed: its counters came
    from other codewords."""
    from ldpc_error_floor_amd import fer
    dec = _make_decoder()
    ck = str(tmp_path / "c.ckpt")
    monkeypatch.setattr(fer, "CHANNEL_STREAM", "philox4x32-10/qms-box-muller")
    with pytest.raises(Stop):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, checkpoint=ck, checkpoint_every=1,
                  progress=_interrupt_after(2))
    monkeypatch.undo()
    assert json.load(open(ck))["key"]["channel"] == "philox4x32-10/qms-box-muller"
    with pytest.raises(ValueError, match="checkpoint is for"):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, checkpoint=ck, resume=True)


def test_old_checkpoint_version_refused(tmp_path):
    ck = tmp_path / "old.ckpt"
    ck.write_text(json.dumps({"version": 1, "key": {}, "si": 0, "pos": 0, "counters": []}))
    with pytest.raises(ValueError, match="checkpoint version 1"):
        fer_sweep(_make_decoder(), SIGMAS, N_CW, BATCH, checkpoint=str(ck), resume=True)


def test_point_seeds_decouple_points_from_their_position():
    """point_seeds: a point's stream is the caller's, not its index in the list (a sweep of one
    SNR run twice with different seeds decodes different noise; with the default seeding the
    first point of any call would reuse seed + 0)."""
    dec = _make_decoder()
    a = _tuples(fer_sweep(dec, SIGMAS[1:], N_CW, BATCH, seed=1076))
    b = _tuples(fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076, point_seeds=[1076, 1076]))
    c = _tuples(fer_sweep(dec, SIGMAS[1:], N_CW, BATCH, point_seeds=[1076 + 7919]))
    d = _tuples(fer_sweep(dec, SIGMAS, N_CW, BATCH, seed=1076))
    assert b[1] == a[0] and c[0] == d[1]
    with pytest.raises(ValueError):
        fer_sweep(dec, SIGMAS, N_CW, BATCH, point_seeds=[1])
