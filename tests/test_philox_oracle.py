"""The channel oracle (oracle/philox_oracle.py) on CPU: Random123 known-answer vectors for
Philox4x32-10, the counter-based streams' sharding property, the Box-Muller channel's
statistics, and the QMS level sampler's level probabilities against create_mix_epoch's model
(Print_Functions.py:29-72) — exactly computed and as the reference's own host channel draws it."""
import numpy as np
import pytest

from oracle.philox_oracle import (awgn_llr, awgn_normals, awgn_q8, awgn_qms_levels, awgn_qms_llr,
                                  near_boundary, philox4x32_10, qms_levels)

# Random123 kat_vectors, philox4x32 with 10 rounds: (counter, key) -> output
KAT = [((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
        (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
       ((0xffffffff, 0xffffffff, 0xffffffff, 0xffffffff), (0xffffffff, 0xffffffff),
        (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
       ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
        (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]


@pytest.mark.parametrize("ctr,key,out", KAT)
def test_philox_known_answers(ctr, key, out):
    got = philox4x32_10(np.array(ctr, np.uint32)[None], key)[0]
    assert [int(x) for x in got] == list(out)


def test_stream_is_indexed_by_global_codeword():
    whole = awgn_normals(40, 101, seed=(1 << 40) + 9, offset=1000)
    part = awgn_normals(15, 101, seed=(1 << 40) + 9, offset=1025)
    assert np.array_equal(whole[25:], part)
    other = awgn_normals(40, 101, seed=(1 << 40) + 10, offset=1000)
    assert not np.array_equal(whole, other)


def test_normal_moments_and_tails():
    x = awgn_normals(2000, 576, seed=1076).astype(np.float64).ravel()
    assert abs(x.mean()) < 0.005 and abs(x.std() - 1) < 0.005
    # 53-bit u1: the largest |n| of 1.15M draws reaches the expected ~5 sigma
    assert 4.5 < np.abs(x).max() < 8.7


def test_channel_model_qms_puncture_shorten():
    sigma = 0.7943282
    llr, raw = awgn_llr(64, 1280, sigma, seed=3, decoding_type=2, q_bit=5, punct=(1, 128),
                        short=(513, 640))
    assert raw is None
    assert np.all(llr[:, :128] == 0) and np.all(llr[:, 512:640] == -20)
    body = llr[:, 128:512]
    assert np.array_equal(body * 2, np.round(body * 2)) and np.abs(body).max() <= 7.5
    # the unquantized LLR of the all-zero word (float modes) has mean -2/sigma^2 and std 2/sigma
    ms, raw = awgn_llr(64, 1280, sigma, seed=3, decoding_type=1)
    r = raw.astype(np.float64)
    assert abs(r.mean() + 2 / sigma ** 2) < 0.02 and abs(r.std() / (2 / sigma) - 1) < 0.01
    sp, _ = awgn_llr(4, 1280, sigma, seed=3, decoding_type=0, punct=(1, 128))
    assert np.all(sp[:, :128] == np.float32(0.001))
    assert near_boundary(np.array([0.25, 0.2500001, 0.3]), 5).tolist() == [True, True, False]


def _level_probs(sigma, q):
    """Exact level probabilities of Cal_MSA_Q(2 (sigma n - 1) / sigma^2), from scipy's ndtr."""
    from scipy.special import ndtr
    T, vals, _ = qms_levels(sigma, q)
    cdf = np.r_[0.0, T.astype(np.float64) / 2.0 ** 64, 1.0]
    return vals, np.diff(cdf), ndtr


@pytest.mark.parametrize("q", [6, 5, -5, 4, 3])
def test_qms_levels_are_cal_msa_q_of_the_channel(q):
    """The thresholds are the CDF of the channel LLR at Cal_MSA_Q's rounding boundaries: each
    level's probability equals P(Q(LLR) = level) computed independently (scipy ndtr on the
    quantizer's own preimage), to float64 precision."""
    from ldpc_error_floor_amd.channel import quantize_host
    sigma = 0.61
    vals, p, ndtr = _level_probs(sigma, q)
    # preimage of each level on a fine LLR grid through the reference's quantizer
    x = np.linspace(-40, 40, 2_000_001)
    qx = quantize_host(x, q)
    for lv, pv in zip(vals, p):
        sel = np.flatnonzero(qx == lv)
        lo, hi = x[sel[0]], x[sel[-1]]
        n_lo = (lo * sigma ** 2 / 2 + 1) / sigma
        n_hi = (hi * sigma ** 2 / 2 + 1) / sigma
        ref = ndtr(n_hi) - ndtr(n_lo)
        assert abs(pv - ref) < 2e-4 * max(ref, 1e-12) + 1e-5, (lv, pv, ref)
    assert abs(p.sum() - 1) < 1e-15


def test_qms_sampler_matches_reference_channel_frequencies():
    """Level frequencies of the sampler (2^21 draws) against the reference's own host channel
    (create_mix_epoch, numpy RandomState) on the same workload (wman, 3.5 dB): both within
    5 sigma of the exact probabilities."""
    from ldpc_error_floor_amd.channel import create_mix_epoch
    sigma, B = 0.5453839, 3600
    vals, p, _ = _level_probs(sigma, 5)
    lv = awgn_qms_levels(B, 576, sigma, seed=1076).ravel()
    X, _ = create_mix_epoch([sigma], np.random.RandomState(2044), np.random.RandomState(1076), B,
                            24, 18, 24, [], True, 2, 0, 0, 0, 0, 5, 20.0)
    ref = np.searchsorted(vals, X.reshape(-1).astype(np.float32))
    n = lv.size
    for counts in (np.bincount(lv, minlength=vals.size), np.bincount(ref, minlength=vals.size)):
        sd = np.sqrt(n * p * (1 - p)) + 1
        assert np.all(np.abs(counts - n * p) < 5 * sd)


def test_qms_stream_sharding_and_layout():
    """Global-codeword indexing (any offset, unaligned quads included) and the byte layout of
    the bytes the bit-sliced kernels' prologue generates per variable and codeword (gen_bytes,
    ldpc_bs_kernel.h) before packing them into planes."""
    sig, seed = 0.7, (1 << 35) + 5
    whole = awgn_qms_llr(77, 130, sig, seed, offset=1001)
    for off in (1002, 1004, 1037):
        part = awgn_qms_llr(77 - (off - 1001), 130, sig, seed, offset=off)
        assert np.array_equal(whole[off - 1001:], part)
    q8 = awgn_q8(70, 130, sig, seed, offset=1001, punct=(1, 3), short=(120, 130))
    assert q8.shape == (3, 130, 32)
    full = awgn_qms_llr(96, 130, sig, seed, offset=1001, punct=(1, 3), short=(120, 130))
    grid = np.rint(full / 0.5).astype(np.int64)
    rows = q8.transpose(0, 2, 1).reshape(96, 130).astype(np.int64)
    assert np.array_equal(rows[:, 3:119] - 16, grid[:, 3:119])
    assert np.all(rows[:, :3] == 16) and np.all(rows[:, 119:] == 48 - 15)


def tie_sigmas(n_vars, seed, offset, q_bit=5, D=1 << 20, bmin=0):
    """Two channel sigmas at which the lowest QMS threshold T_0 shares its high word with the
    uniform U of one element (codeword b >= bmin of offset .. offset + 3, variable v): T_0 = U + ~D
    (level 0) and T_0 = U - ~D (level 1), so that the level rides on the low words.  T_0 falls
    as sigma rises (its boundary is negative), so both come from bisection on sigma; D keeps
    them clear of a last-ulp difference between the host's and the oracle's erfc.
    Returns (b, v, sigma_level0, sigma_level1)."""
    from oracle.philox_oracle import _qms_uniforms, qms_levels
    T0 = lambda s: int(qms_levels(s, q_bit)[0][0])           # noqa: E731
    U = _qms_uniforms(4, n_vars, seed, offset)
    lo_s, hi_s = 0.6, 1.2
    b, v = next((b, v) for b in range(bmin, 4) for v in range(n_vars)
                if T0(hi_s) + 2 * D < int(U[b, v]) < T0(lo_s) - 2 * D
                and 2 * D < (int(U[b, v]) & 0xFFFFFFFF) < (1 << 32) - 2 * D)
    u = int(U[b, v])

    def sigma_at(target):
        a, c = lo_s, hi_s                                     # T0(a) > target >= T0(c)
        for _ in range(80):
            m = 0.5 * (a + c)
            if T0(m) > target:
                a = m
            else:
                c = m
        return a, c

    s0 = sigma_at(u + D)[0]            # T_0 just above U + D: U < T_0, level 0
    s1 = sigma_at(u - D)[1]            # T_0 at most U - D: U >= T_0, level >= 1
    return b, v, s0, s1


def test_qms_high_word_ties_resolve_on_the_low_word():
    """The sampler's 64-bit comparison: at both tie sigmas T_0 and U share the high word (the
    device's first pass stops there and draws the 'LDQR' word), and the level is 0 or 1 as the
    low words order them (the GPU side: tests/test_gpu_channel.py)."""
    from oracle.philox_oracle import _qms_uniforms, qms_levels
    seed, off = 7, 4096
    b, v, s0, s1 = tie_sigmas(576, seed, off)
    u = int(_qms_uniforms(4, 576, seed, off)[b, v])
    for s, lv in ((s0, 0), (s1, 1)):
        t0 = int(qms_levels(s, 5)[0][0])
        assert t0 >> 32 == u >> 32 and t0 != u
        assert awgn_qms_levels(4, 576, s, seed, off)[b, v] == lv
