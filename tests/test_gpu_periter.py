"""Per-iteration parity of the kernels that are actually timed (GPU only).

The reference computes every iteration's hard decisions and syndromes
(``Main_Functions.py:180-209``, ``:317-335``, ``:380-383``) and ``calc_ber_fer`` scores each
iteration's frames (``Print_Functions.py:100-118``).  The throughput path (bench, fer_sweep,
Session counters) runs the bit-sliced kernels bsl / bsc, whose counters-only build exports
``iter_wrong`` (per frame and iteration: a hard decision 1 among the target bits) and whose
export build also stores every iteration's hard decisions (``hard_bits`` / ``synd_bits``).
Both are checked here against the reference fixtures at every iteration, on every exact fixture
the bit-sliced kernels serve (systematic output included), and ``iter_wrong`` of every kernel
against the fixtures / flood."""
import numpy as np
import pytest

from conftest import DECODER_CASES, load_case

pytestmark = pytest.mark.gpu

# exact QMS fixtures whose counters-only decode the bit-sliced kernels must serve
BITSLICED = {"wman_303_q5_snr2.0": "bsl[", "wman_303_q5_snr2.5": "bsl[", "wman_303_q5_snr3.5": "bsl[",
             "wman_303_sys_q5_snr2.5": "bsl[", "wifi_333_q5_snr3.0": "bsl[",
             "g5bg2_222_q5_snr2.0": "bsl[", "g5bg2_222_sys_q5_snr1.75": "bsl[",
             "g5bg1_303_flat_t50_snr2.5": "bsc[", "g5bg1_303_q5_snr3.0": "bsc["}


def _decoder(c, device, kernel="auto"):
    from ldpc_error_floor_amd.decoder import NMSDecoder
    Nt = c["Nt"] if c["Nt"] < c["g"].N else 0
    return NMSDecoder(c["g"].proto, c["z"], c["W"], c["dt"], c["q"], target_node=Nt,
                      device=device, kernel=kernel)


def _wrong_per_iteration(app):
    """[T, B] frame has a hard decision 1 among the output bits (calc_ber_fer per iteration)."""
    return (np.asarray(app) >= 0).any(axis=2)


def test_bitsliced_fixture_set_is_routed_as_expected(cuda_device):
    for name, prefix in BITSLICED.items():
        assert name in DECODER_CASES, name
        dec = _decoder(load_case(name), cuda_device)
        assert dec.kernel_info()[1].startswith(prefix), (name, dec.kernel_info())


@pytest.mark.parametrize("name", sorted(BITSLICED))
def test_bitsliced_every_iteration_matches_reference(name, cuda_device):
    from ldpc_error_floor_amd.decoder import unpack_bits
    c = load_case(name)
    assert c["exact"]
    B = c["llr"].shape[0]
    dec = _decoder(c, cuda_device)
    # export build: every iteration's hard decisions (all N z bits) and syndromes
    res = dec.decode(c["llr"], app=False, hard=True, synd=True, iter_wrong=True, counters=True,
                     flags=True)
    assert dec.last_kernel().startswith(BITSLICED[name]), dec.last_kernel()
    hard = unpack_bits(res.hard.cpu().numpy(), dec.n_vars)
    synd = unpack_bits(res.synd.cpu().numpy(), dec.n_checks)
    for t in range(c["T"]):
        assert np.array_equal(hard[t], c["hard"][t]), (name, t, int((hard[t] != c["hard"][t]).sum()))
        assert np.array_equal(synd[t], c["synd"][t]), (name, t)
    want = _wrong_per_iteration(c["app"])
    assert np.array_equal(res.frame_errors(B), want)
    from _helpers import counters_from_app, flags_from_app
    assert np.array_equal(res.counters.cpu().numpy(), counters_from_app(c["app"]))
    assert np.array_equal(res.flags.cpu().numpy(), flags_from_app(c["app"]))
    # the counters-only build (the one bench.py and fer_sweep time): the same per-iteration
    # frame errors, counters and flags
    r2 = dec.decode(c["llr"], app=False, iter_wrong=True, counters=True, flags=True)
    assert dec.last_kernel() == dec.kernel_info()[1]
    assert np.array_equal(r2.frame_errors(B), want)
    assert np.array_equal(r2.counters.cpu().numpy(), counters_from_app(c["app"]))
    assert np.array_equal(r2.flags.cpu().numpy(), flags_from_app(c["app"]))


@pytest.mark.parametrize("kernel", ["flood", "fused"])
@pytest.mark.parametrize("name", DECODER_CASES)
def test_iter_wrong_every_kernel(name, kernel, cuda_device):
    """iter_wrong of flood, v5 (APP export build), ffl (float modes) and bsl / bsc: equal to the
    fixture's per-iteration frame errors (exact modes) or to flood's (float modes)."""
    c = load_case(name)
    dec = _decoder(c, cuda_device, kernel)
    if not dec.supports(kernel):
        pytest.skip(f"{name}: the {kernel} kernel does not support this configuration")
    B = c["llr"].shape[0]
    counters_only = dec.decode(c["llr"], app=False, iter_wrong=True)
    got = counters_only.frame_errors(B)
    # float modes and q = 6: the fused kernel is the counters-only ffl (no APP export)
    float_mode = c["dt"] in (0, 1, 3) or (c["dt"] == 2 and c["q"] == 6)
    if c["exact"]:
        assert np.array_equal(got, _wrong_per_iteration(c["app"])), dec.last_kernel()
        if kernel == "fused" and not float_mode:
            full = dec.decode(c["llr"], app=True, iter_wrong=True)          # v5 with APP export
            assert dec.last_kernel().startswith("fused5["), dec.last_kernel()
            assert np.array_equal(full.frame_errors(B), _wrong_per_iteration(c["app"]))
    else:
        ref = _decoder(c, cuda_device, "flood").decode(c["llr"], app=True, iter_wrong=True)
        assert np.array_equal(ref.frame_errors(B), _wrong_per_iteration(ref.app.cpu().numpy()))
        assert np.array_equal(got, ref.frame_errors(B)), dec.last_kernel()


def test_bitsliced_export_off_grid_packs(cuda_device):
    """Hard-bit export through bsl with packs off the quantizer grid: those packs are decoded
    by the v5 fixup (its export build), the others by bsl; both halves must equal flood."""
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    proto, g, W, cp = bench.load_problem(T=12, config="C2")
    dec = NMSDecoder(proto, 24, W, 2, 5, device=cuda_device)
    llr = dec.awgn(200, float(cp.sigma(2.0)), seed=3)
    llr[40, 3] += 0.1                 # pack 1 off the grid
    llr[199, 0] = 25.0                # the last (ragged) pack out of range
    # first fill the context's tile buffer with another batch's bits (a v5 APP + hard-bit
    # export): the bit-sliced export does not zero it, its fixup clears the blocks it decodes
    dec.decode(dec.awgn(200, float(cp.sigma(0.5)), seed=4), app=True, hard=True, kernel="fused")
    res = {}
    for k in ("flood", "fused"):
        r = dec.decode(llr, app=False, hard=True, synd=True, iter_wrong=True, kernel=k)
        res[k] = [x.cpu().numpy() for x in (r.hard, r.synd, r.iter_wrong)]
        if k == "fused":
            assert dec.last_kernel().startswith("bsl["), dec.last_kernel()
    for a, b in zip(res["fused"], res["flood"]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("config", ["C2", "C3", "C4", "C5"])
def test_iter_wrong_full_batch_matches_flood(config, cuda_device):
    """B = 2^20 (the bench batch): the timed counters-only kernel's per-iteration frame errors
    equal flood's at every iteration, and fold to its counters."""
    import torch
    import bench
    from ldpc_error_floor_amd.decoder import NMSDecoder
    B = 1 << 20
    cfg = bench.CONFIGS[config]
    proto, g, W, cp = bench.load_problem(config=config)
    dec = NMSDecoder(proto, cfg["z"], W, 2, 5, device=cuda_device, B_max=B)
    punct, short = cfg.get("punct", (0, 0)), cfg.get("short", (0, 0))
    llr = dec.awgn(B, float(cp.sigma(cfg["snr"] - 1.0)), seed=41, punct=punct, short=short)
    out = {}
    for k in ("fused", "flood"):
        r = dec.decode(llr, app=False, iter_wrong=True, counters=True, kernel=k)
        out[k] = (r.iter_wrong.cpu().numpy(), r.counters.cpu().numpy())
        if k == "fused":
            assert dec.last_kernel().startswith(("bsl[", "bsc[")), dec.last_kernel()
        torch.cuda.synchronize()
    assert np.array_equal(out["fused"][0], out["flood"][0])
    w = out["fused"][0].view(np.uint32)
    wrong = np.unpackbits(w.view(np.uint8), bitorder="little").reshape(w.shape[0], -1)[:, :B]
    assert wrong[-1].sum() == out["fused"][1][1]                     # frames wrong at T-1
    assert wrong.all(axis=0).sum() == out["fused"][1][2]            # wrong at every iteration
    assert 0 < wrong[0].sum() and wrong[-1].sum() < wrong[0].sum()
    del llr
    torch.cuda.empty_cache()
