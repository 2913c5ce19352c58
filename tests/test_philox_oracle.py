"""The Philox / Box-Muller channel oracle (oracle/philox_oracle.py) on CPU: Random123
known-answer vectors for Philox4x32-10, the counter-based stream's sharding property, and the
channel statistics of create_mix_epoch's model (Print_Functions.py:29-72)."""
import numpy as np
import pytest

from oracle.philox_oracle import awgn_llr, awgn_normals, near_boundary, philox4x32_10

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
    assert np.all(llr[:, :128] == 0) and np.all(llr[:, 512:640] == -20)
    body = llr[:, 128:512]
    assert np.array_equal(body * 2, np.round(body * 2)) and np.abs(body).max() <= 7.5
    # the unquantized LLR of the all-zero word has mean -2/sigma^2 and std 2/sigma
    r = raw.astype(np.float64)
    assert abs(r.mean() + 2 / sigma ** 2) < 0.02 and abs(r.std() / (2 / sigma) - 1) < 0.01
    sp, _ = awgn_llr(4, 1280, sigma, seed=3, decoding_type=0, punct=(1, 128))
    assert np.all(sp[:, :128] == np.float32(0.001))
    assert near_boundary(np.array([0.25, 0.2500001, 0.3]), 5).tolist() == [True, True, False]
