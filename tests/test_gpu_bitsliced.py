"""The bit-sliced fused kernel (csrc/ldpc_bs.hip: 32 codewords per 32-bit word) that serves
counters-only QMS decodes (GPU only).  Its counters and per-frame flags must equal the flood
kernel's (pinned to the reference fixtures) bit for bit: on ragged batches, with per-row /
per-column weights, for q = 5, -5, 4 and 3, and with LLRs off the quantizer grid (those packs
are decoded by the v5 kernel instead, so the result stays exact for any input)."""
import os

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
DATA = os.path.join(ROOT, "ldpc_error_floor_amd", "data")


def _wman(device, sharing=(3, 0, 3), q=5, T=20, seed=3):
    from ldpc_error_floor_amd.code import CodeParams, TannerGraph, load_base_graph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights, read_weight_file
    proto = load_base_graph(os.path.join(DATA, "BaseGraph", "wman_N0576_R34_z24.txt"))
    g = TannerGraph(proto, 24)
    if sharing == (3, 0, 3):
        wf = read_weight_file(os.path.join(DATA, "Weights",
                                           "C0_wman_N0576_R34_z24_Opt_Weight_End20.txt"))
        W = expand_weights(sharing, {0: wf.blocks[0], 2: wf.blocks[2]}, T, g)
    else:
        rng = np.random.RandomState(seed)
        rows = {0: rng.uniform(0.5, 1.2, (T, g.M)), 2: rng.uniform(0.6, 1.3, (T, g.N))}
        W = expand_weights(sharing, rows, T, g)
    return NMSDecoder(proto, 24, W, 2, q, device=device), CodeParams(proto, 24)


def _both(dec, llr):
    """Counters and flags of flood and of the fused (bit-sliced) counters-only kernel; their
    per-iteration frame-error words must agree too."""
    out, iw = {}, {}
    for k in ("flood", "fused"):
        r = dec.decode(llr, app=False, counters=True, flags=True, kernel=k, iter_wrong=True)
        out[k] = (r.counters.cpu().numpy(), r.flags.cpu().numpy())
        iw[k] = r.iter_wrong.cpu().numpy()
    assert np.array_equal(iw["fused"], iw["flood"]), dec.last_kernel()
    return out


@pytest.fixture(params=["2", "4"], ids=["lpc2", "lpc4"])
def lpc(request, monkeypatch):
    """Both check-lane layouts (2 or 4 lanes per check, LDPC_BS_LPC)."""
    monkeypatch.setenv("LDPC_BS_LPC", request.param)
    return int(request.param)


@pytest.mark.parametrize("B", [1, 31, 33, 3001, 40000])
def test_bitsliced_equals_flood(cuda_device, B, lpc):
    dec, cp = _wman(cuda_device)
    assert dec.kernel_info()[1].endswith(f",l{lpc}]"), dec.kernel_info()
    assert dec.kernel_info()[1].startswith("bsl"), dec.kernel_info()
    llr = dec.awgn(B, float(cp.sigma(2.0)), seed=7, offset=123)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])


@pytest.mark.parametrize("q", [5, -5])
def test_bitsliced_per_row_weights(cuda_device, q, lpc):
    dec, cp = _wman(cuda_device, sharing=(2, 0, 2), q=q, T=12)
    assert dec.kernel_info()[1].startswith("bsl")
    llr = dec.awgn(9000, float(cp.sigma(2.25)), seed=11)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    assert 0 < out["fused"][0][1] < 9000


def test_off_grid_packs_fall_back_exactly(cuda_device, lpc):
    import torch
    dec, cp = _wman(cuda_device)
    llr = dec.awgn(5000, float(cp.sigma(2.0)), seed=9)
    llr[40, 3] += 0.1            # pack 1 off the grid
    llr[4000:4010, 100] = 30.0   # pack 125 out of the quantizer range
    llr[4999, 0] = -0.3          # the last (ragged) pack
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    torch.cuda.synchronize()


def test_off_grid_packs_many_blocks_per_fixup_workgroup(cuda_device):
    """The v5 fixup walks more blocks than its grid has workgroups (k_fused5_fix: 512
    workgroups, each taking the flags of 64 of its blocks per ballot): 2^20 codewords are 65,536
    v5 blocks of 16, 128 per workgroup in two ballots; off-grid packs on several lanes of both of
    one workgroup's ballots (blocks 5 + 512 k), in both halves of a pack, and the last pack."""
    import torch
    dec, cp = _wman(cuda_device)
    B = 1 << 20
    llr = dec.awgn(B, float(cp.sigma(2.5)), seed=21)
    for k in (0, 1, 7, 63, 64, 100, 127):
        llr[16 * (5 + 512 * k) + 3, 10 + k] += 0.1       # block 5 + 512 k
    llr[16 * 1023 + 15, 0] = 40.0                        # the second block of a pack
    llr[B - 1, 5] = -0.2
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    torch.cuda.synchronize()


# ---- the large / UCN instances: 802.11n (C3: degree 22, [3,3,3] UCN, T=50) and 5G BG2 (C4:
# 1,280 variables, [2,2,2] UCN per row and column, puncture and shortening) --------------------
def _config(device, cfg, T=None, ucn_scale=None):
    """A SURVEY workload's decoder; ``ucn_scale``: alpha' = alpha x scale instead of the trained
    alpha' (C4's trained alpha' equals its alpha, which every kernel folds into a decoder without
    UCN: scaling keeps the UCN path of the 5G BG2 instance under test)."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    proto, g, W, cp = bench.load_problem(T=T, config=cfg)
    if ucn_scale is not None:
        W.alpha_ucn = (W.alpha * np.float32(ucn_scale)).astype(np.float32)
    dec = NMSDecoder(proto, g.z, W, 2, 5, device=device)
    c = bench.CONFIGS[cfg]
    dec.punct = c.get("punct", (0, 0))
    dec.short = c.get("short", (0, 0))
    return dec, cp, c


@pytest.mark.parametrize("cfg,T,B,lpc", [("C3", 50, 3001, "4"), ("C3", 12, 40000, "4"),
                                         ("C4", 20, 3001, "4"), ("C4", 20, 3001, "2"),
                                         ("C4", 8, 40000, "4")])
def test_bitsliced_large_and_ucn(cuda_device, cfg, T, B, lpc, monkeypatch):
    monkeypatch.setenv("LDPC_BS_LPC", lpc)
    # (C4's trained alpha' equals its alpha and C3's does for t < 20: both fold to decoders
    # without UCN unless alpha' is scaled)
    dec, cp, c = _config(cuda_device, cfg, T, ucn_scale=0.8 if (cfg == "C4" or T <= 20) else None)
    name = dec.kernel_info()[1]
    assert name.startswith("bsl") and ",ucn" in name, name
    if cfg == "C3":
        # 802.11n (z = 27): column-aligned variable lanes, each column on a half-wave of its own
        # (648 variables on 12 waves instead of 11 packed ones; ldpc_bs.hip colalign_fits)
        assert name.startswith("bsl[p32,w12,"), name
    # (C4 at T = 8 fails every frame 0.75 dB below its point: 0.5 dB above it instead)
    llr = dec.awgn(B, float(cp.sigma(c["snr"] + (0.5 if T < 12 else -0.75))), seed=5, offset=77)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0]), (out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    assert 0 < out["fused"][0][1] < B
    # shortened bits (LLR = -clip_LLR) are decoded in the bit-sliced kernel itself: with the v5
    # fixup switched off the result is unchanged
    monkeypatch.setenv("LDPC_BS_FIXUP", "0")
    r = dec.decode(llr, app=False, counters=True, flags=True, kernel="fused")
    assert np.array_equal(r.counters.cpu().numpy(), out["flood"][0])


def test_identity_ucn_weights_fold(cuda_device):
    """C4's trained alpha' equals its alpha at every iteration, so the unsatisfied-check
    weighting is the identity and ldpc_weights_set folds it away (no ",ucn" kernel): counters and
    flags still equal flood's, and the APP equals the oracle's decode, which applies the UCN
    selection of Main_Functions.py:266-304 with the trained alpha'."""
    from oracle import nms_oracle
    dec, cp, c = _config(cuda_device, "C4", 20)
    assert ",ucn" not in dec.kernel_info()[1], dec.kernel_info()
    llr = dec.awgn(3001, float(cp.sigma(c["snr"] - 0.75)), seed=5, offset=77,
                   punct=c["punct"], short=c["short"])
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    W = dec.weights
    x = llr[:48].cpu().numpy()
    o = nms_oracle.decode(x, dec.graph.proto, 64, W.alpha, W.alpha_ucn, W.beta, 20, 2, 5)
    app = dec.decode(llr[:48], app=True).app.cpu().numpy()
    assert np.array_equal(app, o["app"])


def test_bitsliced_ucn_off_grid_fixup(cuda_device, lpc):
    dec, cp, c = _config(cuda_device, "C4", 10, ucn_scale=0.8)
    assert dec.kernel_info()[1].startswith("bsl"), dec.kernel_info()
    llr = dec.awgn(2000, float(cp.sigma(1.5)), seed=9)
    llr[40, 3] += 0.1            # pack 1 off the grid
    llr[1999, 700] = 9.0         # the last (ragged) pack out of the quantizer range
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])


# ---- the compressed bit-sliced kernel (csrc/ldpc_bsc.hip): 5G BG1 (C5: flat [3,0,3], T=50,
# puncture 1-144, shortening 1537-1584), whose per-edge slots do not fit the LDS --------------
# (T = 12 at 3 dB: about 40 % of the frames fail in the oracle; at 1.75 dB every one does)
@pytest.mark.parametrize("T,B,snr", [(50, 3001, 2.0), (12, 40000, 3.0), (50, 33, 2.5)])
def test_bitsliced_compressed_bg1(cuda_device, T, B, snr, monkeypatch):
    dec, cp, c = _config(cuda_device, "C5", T)
    name = dec.kernel_info()[1]
    assert name.startswith("bsc["), name
    llr = dec.awgn(B, float(cp.sigma(snr)), seed=21, offset=3)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0]), (out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    if B > 1000:
        assert 0 < out["fused"][0][1] < B
    monkeypatch.setenv("LDPC_BS_FIXUP", "0")       # shortened bits decoded in the kernel itself
    r = dec.decode(llr, app=False, counters=True, flags=True, kernel="fused")
    assert np.array_equal(r.counters.cpu().numpy(), out["flood"][0])


def test_bitsliced_compressed_trained_weights(cuda_device):
    """Per-row alpha tables and a trained per-iteration beta (not the flat identity beta) on BG1
    (per-column beta tables do not fit its LDS beside the compressed state: v5 serves those)."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights
    proto, g, _, cp = bench.load_problem(T=10, config="C5")
    rng = np.random.RandomState(4)
    W = expand_weights((2, 0, 3), {0: rng.uniform(0.5, 1.0, (10, g.M)),
                                   2: rng.uniform(0.7, 1.3, (10, 1))}, 10, g)
    dec = NMSDecoder(proto, 72, W, 2, 5, device=cuda_device)
    dec.punct, dec.short = (1, 144), (1537, 1584)
    assert dec.kernel_info()[1].startswith("bsc["), dec.kernel_info()
    llr = dec.awgn(2000, float(cp.sigma(2.0)), seed=8)
    llr[5, 17] += 0.1                              # one pack off the grid (v5 fixup)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])


def test_table_cache_follows_weights_and_T(cuda_device):
    """The per-decode weight / address tables are cached per (weights, T, layout): new weights
    or another T on the same decoder must give what a fresh decoder gives (bsl, bsc, v5)."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import flat_weights
    for cfg in ("C2", "C5"):
        proto, g, W, cp = bench.load_problem(T=12, config=cfg)
        c = bench.CONFIGS[cfg]
        W2 = flat_weights(g, 12, alpha=0.625, beta=1.0)
        dec = NMSDecoder(proto, c["z"], W, 2, 5, device=cuda_device)
        dec.punct, dec.short = c.get("punct", (0, 0)), c.get("short", (0, 0))
        llr = dec.awgn(3000, float(cp.sigma(c["snr"] - 1.0)), seed=6)
        for k in ("fused", "flood"):
            a1 = dec.decode(llr, app=False, counters=True, kernel=k).counters.cpu().numpy()
            a8 = dec.decode(llr, T=8, app=False, counters=True, kernel=k).counters.cpu().numpy()
            dec.set_weights(W2)
            b1 = dec.decode(llr, app=False, counters=True, kernel=k).counters.cpu().numpy()
            dec.set_weights(W)
            c1 = dec.decode(llr, app=False, counters=True, kernel=k).counters.cpu().numpy()
            assert np.array_equal(a1, c1), (cfg, k)
            fresh = NMSDecoder(proto, c["z"], W2, 2, 5, device=cuda_device)
            f1 = fresh.decode(llr, app=False, counters=True, kernel=k).counters.cpu().numpy()
            assert np.array_equal(b1, f1), (cfg, k, b1, f1)
            assert not np.array_equal(a1, b1) and not np.array_equal(a1, a8), (cfg, k)
            if k == "fused":
                ref = {}
                for kk in ("flood",):
                    ref[kk] = dec.decode(llr, T=8, app=False, counters=True, kernel=kk).counters.cpu().numpy()
                assert np.array_equal(a8, ref["flood"]), cfg


@pytest.mark.parametrize("cfg", ["C3", "C4", "C5"])
def test_bitsliced_q_minus5_large_graphs(cuda_device, cfg):
    """q = -5 (grid step 1: shortened bits are +-20 grid units) on the UCN / multi-lane bsl
    instances and on bsc."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    proto, g, W, cp = bench.load_problem(T=10, config=cfg)
    c = bench.CONFIGS[cfg]
    dec = NMSDecoder(proto, c["z"], W, 2, -5, device=cuda_device)
    dec.punct, dec.short = c.get("punct", (0, 0)), c.get("short", (0, 0))
    assert dec.kernel_info()[1].startswith(("bsl[", "bsc[")), dec.kernel_info()
    llr = dec.awgn(2500, float(cp.sigma(c["snr"] - 0.5)), seed=12)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0]), (cfg, out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])


@pytest.mark.parametrize("lpc_c", ["4", "2", "4/2"])
def test_bitsliced_compressed_idle_check_lanes(cuda_device, lpc_c, monkeypatch):
    """bsc with a last check chunk that is only partly used (BG1 lifted by z = 60: 600 checks,
    4 x 600 lanes = 37.5 chunks), where the idle lanes share the last check's record address;
    "4/2": the mixed-lane instance (rows of degree <= 10 at two lanes per check, in chunks of
    their own after the degree-19 rows' chunks, both segments ending in idle lanes)."""
    import bench
    from ldpc_error_floor_amd.code import TannerGraph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import flat_weights
    monkeypatch.setenv("LDPC_BS_LPC", lpc_c.split("/")[0])
    monkeypatch.setenv("LDPC_BSC_MIX", "1" if "/" in lpc_c else "0")
    proto = bench.load_problem(T=10, config="C5")[0]
    g = TannerGraph(proto, 60)
    dec = NMSDecoder(proto, 60, flat_weights(g, 10, alpha=0.75, beta=1.0), 2, 5, device=cuda_device)
    assert dec.kernel_info()[1].startswith("bsc[") and f",l{lpc_c}," in dec.kernel_info()[1], dec.kernel_info()
    from ldpc_error_floor_amd.code import CodeParams
    llr = dec.awgn(3000, float(CodeParams(proto, 60).sigma(3.0)), seed=17)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0]), (out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])


# ---- q = 4 (integers, |v| <= 7) and q = 3 (even integers, |v| <= 6: 3 grid units of 2): the
# messages keep four planes saturated at 15 and the alpha tables are built on min(m, qmax)
# (ldpc_bs.hip, bs_qmax) --------------------------------------------------------------------
@pytest.mark.parametrize("q", [4, 3])
@pytest.mark.parametrize("sharing", [(3, 0, 3), (2, 0, 2)])
def test_bitsliced_q4_q3_wman(cuda_device, q, sharing, lpc):
    dec, cp = _wman(cuda_device, sharing=sharing, q=q, T=20 if sharing == (3, 0, 3) else 12)
    assert dec.kernel_info()[1].startswith("bsl") and dec.kernel_info()[1].endswith(f",l{lpc}]"), \
        dec.kernel_info()
    for B, snr in ((3001, 2.0), (64, 3.0)):
        llr = dec.awgn(B, float(cp.sigma(snr)), seed=21 + B, offset=5)
        out = _both(dec, llr)
        assert np.array_equal(out["fused"][0], out["flood"][0]), (q, out["fused"][0], out["flood"][0])
        assert np.array_equal(out["fused"][1], out["flood"][1])
    assert 0 < out["fused"][0][3] or B == 64


@pytest.mark.parametrize("q", [4, 3])
def test_bitsliced_q4_q3_off_grid(cuda_device, q):
    """On the q = 4 / 3 grids a value of the q = 5 grid (0.5) or beyond qmax (9 > 7, 8 > 6) is
    off the grid: its pack goes to the v5 fixup and the result stays exact."""
    dec, cp = _wman(cuda_device, q=q)
    llr = dec.awgn(3000, float(cp.sigma(2.0)), seed=4)
    llr[40, 3] = 0.5
    llr[1000, 7] = 9.0 if q == 4 else 8.0
    llr[2999, 0] = -1.0 if q == 3 else 1.5
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])


@pytest.mark.parametrize("q", [4, 3])
@pytest.mark.parametrize("cfg", ["C3", "C4", "C5"])
def test_bitsliced_q4_q3_large_graphs(cuda_device, cfg, q, monkeypatch):
    """The UCN / multi-lane bsl instances and bsc on q = 4 / 3: shortened bits are -clip_LLR =
    -20 (20 / 10 grid units > qmax), decoded in place (the v5 fixup switched off gives the same)."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    proto, g, W, cp = bench.load_problem(T=12, config=cfg)
    c = bench.CONFIGS[cfg]
    dec = NMSDecoder(proto, c["z"], W, 2, q, device=cuda_device)
    dec.punct, dec.short = c.get("punct", (0, 0)), c.get("short", (0, 0))
    assert dec.kernel_info()[1].startswith(("bsl[", "bsc[")), dec.kernel_info()
    # (BG1 at T = 12: 0.5 dB above its 3 dB point, where q = 3 still fails ~85 % of the frames)
    llr = dec.awgn(2500, float(cp.sigma(c["snr"] + (0.5 if cfg == "C5" else -0.5))), seed=13)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0]), (cfg, q, out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
    assert 0 < out["fused"][0][1] < 2500
    if c.get("short", (0, 0))[0]:
        monkeypatch.setenv("LDPC_BS_FIXUP", "0")
        r = dec.decode(llr, app=False, counters=True, flags=True, kernel="fused")
        assert np.array_equal(r.counters.cpu().numpy(), out["flood"][0])


def test_bitsliced_more_than_64_iterations(cuda_device):
    """T = 70 with a beta that is the identity on the grid in the first iterations only: the
    identity-table mask covers iterations 0..63 and must not wrap onto later ones."""
    from ldpc_error_floor_amd.code import CodeParams, TannerGraph, load_base_graph
    from ldpc_error_floor_amd.decoder import NMSDecoder
    from ldpc_error_floor_amd.weights import expand_weights
    proto = load_base_graph(os.path.join(DATA, "BaseGraph", "wman_N0576_R34_z24.txt"))
    g = TannerGraph(proto, 24)
    T = 70
    beta = np.where(np.arange(T) < 8, 1.0, 0.7)[:, None]    # identity at t < 8 only: a wrapped
    #                                                         mask would skip t = 64..69's tables
    W = expand_weights((3, 0, 3), {0: np.full((T, 1), 0.75), 2: beta}, T, g)
    dec = NMSDecoder(proto, 24, W, 2, 5, device=cuda_device)
    assert dec.kernel_info()[1].startswith("bsl"), dec.kernel_info()
    llr = dec.awgn(2000, float(CodeParams(proto, 24).sigma(2.0)), seed=8)
    out = _both(dec, llr)
    assert np.array_equal(out["fused"][0], out["flood"][0]), (out["fused"][0], out["flood"][0])
    assert np.array_equal(out["fused"][1], out["flood"][1])
