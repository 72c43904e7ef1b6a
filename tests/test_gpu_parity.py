"""Parity of the HIP path (through the C-ABI) against the CPU oracle and the reference's golden
vectors. Run on an MI355X: python -m pytest tests -m gpu.

Tolerance: relative L2 <= 1e-10 and max-abs <= 1e-10 * max|ref| (fp64),
unless a test states otherwise (bit-exact for Philox words and for batch-split invariance).
"""
import zlib

import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity, rel_err
from tests.helpers import common_signal, oracle_segments, per_psr_signal, random_layout

pytestmark = pytest.mark.gpu

TOL = 1e-10


@pytest.fixture(scope="module")
def capi():
    from fakepta_amd import _capi
    return _capi


@pytest.fixture(scope="module")
def ctx(capi):
    c = capi.Context(0)
    yield c
    c.close()


# ----------------------------------------------------------------------------- RNG
def test_philox_device_bit_exact(ctx):
    kat = np.array([[0, 0, 0, 0], [0xffffffff] * 4, [0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344]], np.uint32)
    keys = [(0, 0), (0xffffffff, 0xffffffff), (0xa4093822, 0x299f31d0)]
    want = [(0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)]
    for c, k, w in zip(kat, keys, want):
        assert tuple(int(x) for x in ctx.debug_philox(c[None], np.array(k, np.uint32))[0]) == w
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2 ** 32, size=(20000, 4), dtype=np.uint64).astype(np.uint32)
    key = np.array([123456789, 987654321], np.uint32)
    np.testing.assert_array_equal(ctx.debug_philox(ctr, key), O.philox4x32_10(ctr, key))


def test_device_normals_match_oracle(ctx):
    """The device's normal map (philox.h normals4: 32-bit Box-Muller with fp64 polynomials) restates the oracle's
    operation for operation: coefficients downloaded from the batch path (amp * z, k_gen) equal the oracle's to
    1e-13 relative, for an even and an odd first realization (the realization-pair straddle)."""
    rng = np.random.default_rng(5)
    offs, toas, nu = random_layout(rng, 3, (30, 60))
    ctx.batch_set_toas(offs, toas, nu)
    f, a = per_psr_signal(rng, offs, toas, 12)
    ctx.batch_add_signal(0, f, a)
    for real0 in (0, 7):
        _, co = ctx.batch_synth(77, real0, 9, coeffs=True)  # [P][K][R]
        for p in range(3):
            z = O.gp_normals(77, np.arange(real0, real0 + 9), p, 0, 12)  # [R, N, 2]
            want = np.transpose(a[p][None, :, None] * z, (1, 2, 0)).reshape(24, 9)
            np.testing.assert_allclose(co[p], want, rtol=1e-13, atol=1e-13 * np.abs(want).max())


def test_device_normals4_edge_words(ctx):
    """The device normal map on chosen words (fpta_debug_normals), not only on Philox outputs: the logarithm word at
    its ends (0: the largest radius; 0xFFFFFFFF: u1 = 1, radius exactly 0 through bm_sqrt's x > 0 select) and around
    2^31; the angle word at every quarter turn (q = 4 wraps to quadrant 0), one below and above, and the rint ties
    between quarter turns; plus 200k random words. Within a few ulp of the oracle's IEEE division / square root (the
    device uses v_rcp_f64 / v_rsq_f64 refinements)."""
    edge_a = np.array([0, 1, 2, 0x7FFFFFFE, 0x7FFFFFFF, 0x80000000, 0x80000001, 0xFFFFFFFD, 0xFFFFFFFE, 0xFFFFFFFF],
                      dtype=np.uint64)
    qb = [k << 30 for k in range(4)] + [(2 * k + 1) << 29 for k in range(4)]
    edge_b = np.unique(np.clip(np.array([b + d for b in qb for d in (-2, -1, 0, 1, 2)] + [0xFFFFFFFF],
                                        dtype=np.int64), 0, 0xFFFFFFFF)).astype(np.uint64)
    a, b = np.meshgrid(edge_a, edge_b, indexing="ij")
    a, b = a.ravel(), b.ravel()
    edges = np.stack([a, b, b[::-1], a[::-1]], 1).astype(np.uint32)
    rng = np.random.default_rng(11)
    words = np.concatenate([edges, rng.integers(0, 2 ** 32, size=(200000, 4), dtype=np.uint64).astype(np.uint32)])
    got = ctx.debug_normals(words)
    want = O.normals4(words)
    assert np.all(np.isfinite(got))
    # error in units of the pair's radius ulp (a cos / sin value near zero is judged against its pair's radius)
    radius = np.repeat(np.hypot(want[:, 0::2], want[:, 1::2]), 2, axis=1)
    ulps = np.abs(got - want) / (np.finfo(np.float64).eps * np.maximum(radius, np.finfo(np.float64).tiny))
    worst = np.unravel_index(np.argmax(ulps), ulps.shape)
    assert ulps.max() <= 16.0, (float(ulps.max()), words[worst[0]].tolist(), float(got[worst]), float(want[worst]))
    zero_r = words[:, 0] == 0xFFFFFFFF
    assert np.all(got[zero_r, :2] == 0.0)


# ----------------------------------------------------------------------------- drop-in kernels vs fixtures
@pytest.mark.parametrize("lab", ["rn", "dm", "sv"])
def test_gp_accumulate_vs_reference(ctx, golden, lab):
    g = golden("g2_single_psr.npz")
    f, psd, z, idx = g[f"{lab}_f"], g[f"{lab}_psd"], g[f"{lab}_z"], float(g[f"{lab}_idx"])
    c = O.gp_coeffs_from_z(psd, z)
    sq = O.delta_f(f) ** 0.5
    r = np.zeros(len(g["toas"]))
    ctx.gp_accumulate(g["toas"], g["freqs"], [(f, sq * c[0::2], sq * c[1::2], idx, 1400.0)], r)
    assert_parity(r, g[f"{lab}_delta"], 1e-12)
    rec = np.zeros_like(r)
    df = O.delta_f(f)
    ctx.gp_accumulate(g["toas"], g["freqs"], [(f, df * g[f"{lab}_fourier"][0], df * g[f"{lab}_fourier"][1], idx,
                                               1400.0)], rec)
    assert_parity(rec, g[f"{lab}_reconstruct"], 1e-12)


def test_dropin_single_pulsar_replay(golden):
    """The reference's own call sequence (tools/gen_golden.py gen_g2) through the fakepta drop-in."""
    from fakepta import fake_pta as fp
    g = golden("g2_single_psr.npz")
    rng = np.random.default_rng(7)
    yr = 365.25 * 24 * 3600
    keep = rng.random(330) < 0.75
    cadence = 12.3 * 24 * 3600
    epochs = 0.35 * yr + np.arange(1, 331)[keep] * cadence
    np.random.seed(11)
    psr = fp.Pulsar(epochs, 3e-7, 1.1, 4.2, pdist=(1.0, 0.2), freqs=[1400], backends=["A.1400", "B.800"],
                    custom_model={"RN": 30, "DM": 100, "Sv": 30})
    for b in psr.backends:
        psr.noisedict[f"{psr.name}_{b}_efac"] = {"A.1400": 1.3, "B.800": 0.8}[b]
        psr.noisedict[f"{psr.name}_{b}_log10_tnequad"] = {"A.1400": -6.5, "B.800": -7.2}[b]
    for lab, call in (("rn", lambda: psr.add_red_noise(spectrum="powerlaw", log10_A=-13.4, gamma=3.3)),
                      ("dm", lambda: psr.add_dm_noise(spectrum="powerlaw", log10_A=-13.1, gamma=2.5)),
                      ("sv", lambda: psr.add_chromatic_noise(spectrum="powerlaw", log10_A=-13.6, gamma=2.0))):
        before = psr.residuals.copy()
        call()
        assert_parity(psr.residuals - before, g[f"{lab}_delta"], 1e-11)
    for sig, lab in (("red_noise", "rn"), ("dm_gp", "dm"), ("chrom_gp", "sv")):
        np.testing.assert_allclose(psr.signal_model[sig]["fourier"], g[f"{lab}_fourier"], rtol=1e-15)
        assert_parity(psr.reconstruct_signal([sig]), g[f"{lab}_reconstruct"], 1e-12)
    assert_parity(psr.residuals, g["total_after_gp"], 1e-12)
    assert_parity(psr.reconstruct_signal(), g["reconstruct_all"], 1e-12)
    psr.add_red_noise(spectrum="powerlaw", log10_A=-13.0, gamma=4.1)  # replace-on-reinject
    assert_parity(psr.residuals, g["rn2_residuals"], 1e-11)
    before = psr.residuals.copy()
    psr.add_white_noise()
    assert_parity(psr.residuals - before, g["wn_delta"], 1e-10)
    # remove_signal returns the residuals to white noise + the remaining GPs
    psr.remove_signal(["red_noise", "dm_gp", "chrom_gp"])
    assert_parity(psr.residuals, g["wn_delta"], 1e-8)


@pytest.mark.parametrize("orf", ["hd", "monopole", "dipole", "curn"])
def test_dropin_common_vs_reference(golden, orf):
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    g = golden("g3_common.npz")
    np.random.seed(5)
    psrs = fp.make_fake_array(npsrs=25, Tobs=None, ntoas=120, gaps=True, toaerr=1e-7, isotropic=True,
                              backends=["A.1400", "B.800"], custom_model={"RN": None, "DM": None, "Sv": None})
    np.testing.assert_array_equal(np.concatenate([p.toas for p in psrs]), g["toas"])
    np.testing.assert_array_equal(np.concatenate([p.freqs for p in psrs]), g["freqs"])
    # replay the fixture generator's ORF loop up to this ORF (the RNG stream is shared)
    for o in ("hd", "monopole", "dipole", "curn"):
        for p in psrs:
            p.make_ideal()
        cn.add_common_correlated_noise(psrs, orf=o, spectrum="powerlaw", name="gw",
                                       idx=2.0 if o == "dipole" else 0, components=30, log10_A=-14.2,
                                       gamma=13 / 3)
        if o == orf:
            break
    fourier = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
    np.testing.assert_allclose(fourier, g[f"{orf}_fourier"], rtol=1e-10, atol=1e-10 * np.abs(fourier).max())
    assert_parity(np.concatenate([p.residuals for p in psrs]), g[f"{orf}_residuals"], TOL)
    assert_parity(np.concatenate([p.reconstruct_signal(["gw_common"]) for p in psrs]), g[f"{orf}_reconstruct"],
                  TOL)
    # the one-launch array reconstruct against the reference's own per-pulsar reconstruct_signal
    assert_parity(np.concatenate(fp.reconstruct_array(psrs, ["gw_common"])), g[f"{orf}_reconstruct"], TOL)


def test_user_orf_matrix_dropin(golden):
    """orf= an ORF matrix (this package accepts any PSD matrix; the reference's string ORFs are the
    named cases): passing the reference's own Hellings-Downs matrix reproduces its orf='hd' injection
    (same draws, same SVD factor), and BatchSimulator on that array equals the named-ORF array bit for bit."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    g = golden("g3_common.npz")
    np.random.seed(5)
    psrs = fp.make_fake_array(npsrs=25, Tobs=None, ntoas=120, gaps=True, toaerr=1e-7, isotropic=True,
                              backends=["A.1400", "B.800"], custom_model={"RN": None, "DM": None, "Sv": None})
    for p in psrs:
        p.make_ideal()
    cn.add_common_correlated_noise(psrs, orf=np.array(g["hd_orf"]), spectrum="powerlaw", name="gw", idx=0,
                                   components=30, log10_A=-14.2, gamma=13 / 3)
    assert_parity(np.concatenate([p.residuals for p in psrs]), g["hd_residuals"], TOL)
    fourier = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
    np.testing.assert_allclose(fourier, g["hd_fourier"], rtol=1e-10, atol=1e-10 * np.abs(fourier).max())
    user = BatchSimulator(psrs, white=False).synth(40, seed=3)
    for p in psrs:
        p.signal_model["gw_common"]["orf"] = "hd"
    named = BatchSimulator(psrs, white=False).synth(40, seed=3)
    np.testing.assert_array_equal(user, named)
    seg = oracle_segments(BatchSimulator(psrs, white=False))
    offs = np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])])
    want = O.batch_synth(offs, np.concatenate([p.toas for p in psrs]), np.concatenate([p.freqs for p in psrs]),
                         seg, 3, 0, 40)
    assert_parity(user, want, TOL)


def test_reference_pickle_session_continues(golden):
    """Pulsars pickled by the reference (fixture g7, class path fakepta.fake_pta.Pulsar) load into the drop-in
    and the session continues as in the reference: reconstruct_signal() of every signal, then a seeded
    replace-on-reinject of the red noise and a second common-signal injection."""
    import os
    import pickle
    from fakepta import correlated_noises as cn
    from tests.conftest import GOLDEN
    g = golden("g7_ref_pulsars.npz")
    with open(os.path.join(GOLDEN, "g7_ref_pulsars.pkl"), "rb") as fh:
        psrs = pickle.load(fh)
    for i, p in enumerate(psrs):
        assert_parity(p.reconstruct_signal(), g[f"reconstruct_all_{i}"], 1e-12)
    np.random.seed(32)
    for p in psrs:
        p.add_red_noise(spectrum="powerlaw", log10_A=-13.5, gamma=3.5)
    cn.add_common_correlated_noise(psrs, orf="hd", components=15, log10_A=-14.0, gamma=4.0)
    for i, p in enumerate(psrs):
        np.testing.assert_allclose(p.signal_model["red_noise"]["fourier"], g[f"rn_fourier_after_{i}"], rtol=1e-15)
        assert_parity(p.residuals, g[f"residuals_after_{i}"], 1e-11)


def test_reference_script_imports_reproduce_g4(golden):
    """examples/make_fake_array.py's own import line and call, BASELINE configs[0] (G4)."""
    from fakepta.fake_pta import make_fake_array
    g = golden("g4_make_fake_array.npz")
    np.random.seed(0)
    psrs = make_fake_array(npsrs=25, Tobs=10, ntoas=1000, isotropic=True, gaps=True, toaerr=1e-7,
                           backends="NUPPI.1400", custom_model={"RN": 30, "DM": None, "Sv": None})
    assert_parity(np.concatenate([p.residuals for p in psrs]), g["residuals"], TOL)


def _g8_workflow(golden):
    """examples/make_fake_array.py:34-47 through the drop-in, on fixture G8's stand-in EPTA pulsars with the
    reference's own noisedict / custom_models JSON."""
    from fakepta.correlated_noises import add_common_correlated_noise
    from fakepta.fake_pta import copy_array
    from tests.helpers import g8_inputs
    psrs_0, nd, cm, g = g8_inputs(golden)
    np.random.seed(int(g["seed"]))
    psrs = copy_array(psrs_0, nd, cm)
    for psr in psrs:
        psr.make_ideal()
        psr.add_white_noise()
        psr.add_red_noise()
        psr.add_dm_noise()
        psr.add_chromatic_noise()
    noise = np.concatenate([p.residuals for p in psrs])
    add_common_correlated_noise(psrs, log10_A=-15., gamma=13 / 3, orf='hd')
    return psrs, g, noise


def test_example_workflow_g8(golden):
    """Fixture G8: copy_array + noisedict-driven add_red_noise() / add_dm_noise() / add_chromatic_noise() with
    ragged per-pulsar mode counts (RN 10-99, DM 11-100, Sv 93, None) and the HD GWB reproduce the reference's
    residuals, signal_model entries and noisedicts."""
    psrs, g, noise = _g8_workflow(golden)
    want = golden("g8_example_workflow.json")
    assert_parity(noise, g["residuals_noise"], TOL)
    assert_parity(np.concatenate([p.residuals for p in psrs]), g["residuals"], TOL)
    for i, p in enumerate(psrs):
        assert p.noisedict == want["noisedicts"][p.name]
        assert sorted(p.signal_model) == sorted(want["signal_models"][p.name])
        for sig, meta in want["signal_models"][p.name].items():
            sm, key = p.signal_model[sig], f"{i}_{sig}"
            assert sm["nbin"] == meta["nbin"] and float(sm["idx"]) == meta["idx"]
            np.testing.assert_array_equal(sm["f"], g[key + "_f"])
            np.testing.assert_array_equal(sm["psd"], g[key + "_psd"])
            tol = 1e-15 if sig != "gw_common" else 1e-10
            np.testing.assert_allclose(sm["fourier"], g[key + "_fourier"], rtol=tol,
                                       atol=tol * np.abs(g[key + "_fourier"]).max())
            assert_parity(p.reconstruct_signal([sig]), g[key + "_reconstruct"], TOL)


@pytest.mark.parametrize("path", [0, 1, 2, 3, 4])
def test_example_workflow_batch_vs_oracle(golden, capi, path):
    """BatchSimulator on the G8 array: per-pulsar signals with ragged mode counts (zero-amplitude padding up
    to the largest), pulsars without a signal, multi-backend white noise, on real-MJD epochs; every synthesis
    path vs the oracle."""
    from fakepta_amd.batch import BatchSimulator
    psrs, _, _ = _g8_workflow(golden)
    sim = BatchSimulator(psrs, white=True)
    assert [s["name"] for s in sim.segments] == ["red_noise", "gw_common", "dm_gp", "chrom_gp"]
    segs = oracle_segments(sim)
    shipped = sim.ctx.options()
    sim.ctx.set_option(capi.OPT_SYNTH_PATH, path)
    try:
        for real0, R in ((0, 24), (70001, 5)):
            got = sim.synth(R, seed=17, real0=real0)
            want = O.batch_synth(sim.offs, sim.toas, sim.freqs, segs, 17, real0, R, sigma=sim.sigma)
            assert_parity(got, want, TOL)
    finally:
        sim.ctx.set_options(shipped)


def test_common_components_not_len_f_g9(golden):
    """Fixture G9 (correlated_noises.py:140-160): with 40 frequencies and components=30 the drop-in injects 30
    modes, stores f / psd with 40 entries and fourier [2, 30], and leaves np.random where the reference does;
    with 20 frequencies it injects them all, draws one more pair and raises the reference's IndexError."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    g = golden("g9_common_components.npz")
    np.random.seed(9)
    psrs = fp.make_fake_array(npsrs=8, Tobs=8, ntoas=90, gaps=True, toaerr=1e-7, isotropic=True,
                              backends=["A.1400", "B.800"], custom_model={"RN": None, "DM": None, "Sv": None})
    np.testing.assert_array_equal(np.concatenate([p.toas for p in psrs]), g["toas"])
    for p in psrs:
        p.make_ideal()
    cn.add_common_correlated_noise(psrs, orf="hd", components=30, f_psd=g["long_f"], log10_A=-14.5, gamma=13 / 3,
                                   idx=2)
    sm = psrs[0].signal_model["gw_common"]
    assert sm["nbin"] == 30 and len(sm["f"]) == 40
    np.testing.assert_array_equal(sm["psd"], g["long_psd"])
    fourier = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
    np.testing.assert_allclose(fourier, g["long_fourier"], rtol=1e-10, atol=1e-10 * np.abs(fourier).max())
    assert_parity(np.concatenate([p.residuals for p in psrs]), g["long_residuals"], TOL)
    assert_parity(np.concatenate([p.reconstruct_signal(["gw_common"]) for p in psrs]), g["long_reconstruct"], TOL)
    assert_parity(np.concatenate(fp.reconstruct_array(psrs, ["gw_common"])), g["long_reconstruct"], TOL)
    np.testing.assert_array_equal(np.random.standard_normal(4), g["long_next_draw"])
    assert BatchSimulator(psrs, white=False).segments[0]["f"].shape == (30,)
    np.random.seed(19)
    for p in psrs:
        p.make_ideal()
    with pytest.raises(IndexError, match=str(g["short_error"])):
        cn.add_common_correlated_noise(psrs, orf="hd", components=30, f_psd=g["long_f"][:20], log10_A=-14.5,
                                       gamma=13 / 3)
    assert_parity(np.concatenate([p.residuals for p in psrs]), g["short_residuals"], TOL)
    fourier = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
    np.testing.assert_allclose(fourier, g["short_fourier"], rtol=1e-10, atol=1e-10 * np.abs(fourier).max())
    np.testing.assert_array_equal(np.random.standard_normal(4), g["short_next_draw"])


def test_reconstruct_array_and_common_reinject():
    """One-launch array reconstruct == per-pulsar reconstruct_signal; re-injecting a common signal
    replaces it (correlated_noises.py:133-134)."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    np.random.seed(12)
    psrs = fp.make_fake_array(npsrs=9, Tobs=None, ntoas=80, gaps=True, toaerr=1e-7, isotropic=False,
                              backends=["A.1400", "B.800"], custom_model={"RN": 20, "DM": 35, "Sv": None})
    psrs[3].custom_model = {"RN": 7, "DM": None, "Sv": 12}
    psrs[3].add_chromatic_noise(log10_A=-13.5, gamma=2.0)
    psrs[4].add_system_noise(backend="B.800", components=9, log10_A=-13.2, gamma=3.0)
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-14.0, gamma=13 / 3, components=25)
    sigs = ["red_noise", "dm_gp", "chrom_gp", "gw_common", "B.800_system_noise_B.800"]
    arr = fp.reconstruct_array(psrs, sigs)
    for p, r in zip(psrs, arr):
        own = [s for s in sigs if s in p.signal_model]
        assert_parity(r, p.reconstruct_signal(own), 1e-12)
    for p in psrs:
        p.make_ideal()
    cn.add_common_correlated_noise(psrs, orf="dipole", log10_A=-14.0, gamma=13 / 3, components=10)
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-13.7, gamma=4.0, components=10)
    rec = fp.reconstruct_array(psrs, ["gw_common"])
    scale = max(np.abs(p.residuals).max() for p in psrs)
    for p, r in zip(psrs, rec):
        np.testing.assert_allclose(p.residuals, r, rtol=0, atol=1e-11 * scale)


@pytest.mark.parametrize("fixture,kwargs", [
    ("g4_make_fake_array.npz", dict(seed=0, npsrs=25, Tobs=10, ntoas=1000, isotropic=True, gaps=True, toaerr=1e-7,
                                    backends="NUPPI.1400", custom_model={"RN": 30, "DM": None, "Sv": None})),
    ("g4b_make_fake_array.npz", dict(seed=1, npsrs=6, Tobs=None, ntoas=None, gaps=True, toaerr=None,
                                     backends=["A.1400", "B.800"], isotropic=False)),
])
def test_make_fake_array_end_to_end(golden, fixture, kwargs):
    """BASELINE configs[0]: seeded make_fake_array reproduces the reference's residuals."""
    from fakepta import fake_pta as fp
    g = golden(fixture)
    kwargs = dict(kwargs)
    np.random.seed(kwargs.pop("seed"))
    psrs = fp.make_fake_array(**kwargs)
    assert [p.name for p in psrs] == list(g["names"])
    np.testing.assert_array_equal(np.concatenate([p.toas for p in psrs]), g["toas"])
    assert_parity(np.concatenate([p.residuals for p in psrs]), g["residuals"], TOL)
    if "rn_fourier" in g:
        np.testing.assert_allclose(np.array([p.signal_model["red_noise"]["fourier"] for p in psrs]), g["rn_fourier"],
                                   rtol=1e-15)


def test_white_ecorr_dropin(ctx):
    rng = np.random.default_rng(3)
    n = 500
    sigma = rng.uniform(1e-7, 1e-6, n)
    z = rng.standard_normal(n)
    blocks = [np.arange(i, min(i + 4, n)) for i in range(0, n, 4)]
    es = rng.uniform(1e-8, 1e-7, len(blocks))
    zb = rng.standard_normal(len(blocks))
    r = rng.normal(size=n) * 1e-6
    want = r + sigma * z
    for b, e, zz in zip(blocks, es, zb):
        want[b] += e * zz
    ctx.white_accumulate(sigma, z, r, blocks=blocks, ecorr_sigma=es, zb=zb)
    assert_parity(r, want, 1e-14)


def test_masked_system_noise(ctx):
    """Backend mask (fake_pta.py:361-368, D9 fixed) and add_system_noise (D3 fixed)."""
    from fakepta import fake_pta as fp
    np.random.seed(4)
    psr = fp.Pulsar(np.linspace(0, 3e8, 200), 1e-7, 0.3, 0.4, backends=["A.1400", "B.800"],
                    custom_model={"RN": None, "DM": None, "Sv": None})
    psr.add_system_noise(backend="B.800", components=12, log10_A=-13.0, gamma=3.0)
    name = "B.800_system_noise_B.800"
    sm = psr.signal_model[name]
    m = psr.backend_flags == "B.800"
    coeffs = np.empty(24)
    df = O.delta_f(sm["f"])
    coeffs[0::2], coeffs[1::2] = sm["fourier"][0] * df ** 0.5, sm["fourier"][1] * df ** 0.5
    want = O.gp_synth_loop(psr.toas, psr.freqs, sm["f"], coeffs, 0.0, mask=m)
    assert_parity(psr.residuals, want, 1e-12)
    assert np.all(psr.residuals[~m] == 0)
    psr.add_system_noise(backend="B.800", components=12, log10_A=-13.0, gamma=3.0)  # replaces, not adds
    assert_parity(psr.reconstruct_signal([name]), psr.residuals, 1e-12)


# ----------------------------------------------------------------------------- batch path vs oracle
def _build(ctx, rng, P=7, n_range=(20, 260), per_psr=((30, 0.0), (41, 2.0)), common=((30, 0.0),), masked=False,
           white=False, ecorr=False):
    offs, toas, nu = random_layout(rng, P, n_range)
    ctx.batch_set_toas(offs, toas, nu)
    segs = []
    for nm, idx in per_psr:
        f, a = per_psr_signal(rng, offs, toas, nm)
        mask = None
        if masked:
            mask = (rng.random(offs[-1]) < 0.5).astype(np.uint8)
        ctx.batch_add_signal(0, f, a, idx=idx, mask=mask)
        segs.append(O.Segment(0, 2 * np.pi * f, a, idx, mask=mask))
    for nm, idx in common:
        f, a, L, _ = common_signal(rng, offs, toas, nm)
        ctx.batch_add_signal(1, f, a, idx=idx, L=L)
        segs.append(O.Segment(1, 2 * np.pi * f, a, idx, L=L))
    sigma = blocks = es = block_of = None
    if white:
        sigma = rng.uniform(1e-7, 1e-6, offs[-1])
    if ecorr:
        starts = np.arange(0, offs[-1], 3)
        blocks = [np.arange(s, min(s + 2, offs[-1])) for s in starts]
        es = rng.uniform(1e-8, 1e-7, len(blocks))
        block_of = -np.ones(offs[-1], dtype=np.int64)
        for b, q in enumerate(blocks):
            block_of[q] = b
    if white or ecorr:
        ctx.batch_set_white(sigma, blocks, es)
    return offs, toas, nu, segs, sigma, block_of, es


PATHS = [(1, 0), (2, 0)] + [(3, v) for v in range(6)] + [(4, 0)]  # (synth path, VALU variant); 4 = gridded


@pytest.mark.parametrize("path,variant", PATHS)
@pytest.mark.parametrize("case", ["basic", "masked_odd_modes", "white_ecorr", "white_only", "ecorr_only",
                                  "common_only", "tiny_pulsars"])
def test_batch_vs_oracle(ctx, capi, path, variant, case):
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    kw = dict(basic={}, masked_odd_modes=dict(per_psr=((7, 4.0), (1, 0.0)), masked=True),
              white_ecorr=dict(white=True, ecorr=True), white_only=dict(white=True, P=3),
              ecorr_only=dict(ecorr=True, per_psr=((12, 0.0),), common=()), common_only=dict(per_psr=(), common=((30, 0.0), (13, 2.0))),
              tiny_pulsars=dict(P=5, n_range=(1, 18)))[case]
    offs, toas, nu, segs, sigma, block_of, es = _build(ctx, rng, **kw)
    shipped = ctx.options()
    ctx.set_option(capi.OPT_SYNTH_PATH, path)
    ctx.set_option(capi.OPT_VALU_VARIANT, variant)
    try:
        for real0, R in ((0, 70), (1000003, 3), (5, 257)):
            got = ctx.batch_synth(99, real0, R)
            want = O.batch_synth(offs, toas, nu, segs, 99, real0, R, sigma=sigma, block_of=block_of,
                                 ecorr_sigma=es)
            assert_parity(got, want, TOL)
    finally:
        ctx.set_options(shipped)


def test_variant_switches_write_every_sample(ctx, capi):
    """Regression for DESIGN.md §10 (the tile table of one kernel must never drive another): replay the
    synthesis sweep's order (MFMA, then every VALU and seeded-VALU variant, then the gridded path, at one
    fixed n_real) with the device block poisoned with NaN before every launch, so a kernel that skips part
    of the block, or reuses a stale tile table, fails here instead of being masked by the previous output."""
    rng = np.random.default_rng(44)
    offs, toas, nu, segs, *_ = _build(ctx, rng, P=6, n_range=(150, 700))
    want = O.batch_synth(offs, toas, nu, segs, 1234, 0, 256)
    shipped = ctx.options()
    order = [(2, 0)] + [(3, v) for v in range(6)] + [(2, 0), (4, 0), (1, 0), (3, 4)]
    try:
        ctx.batch_synth(1234, 0, 256, to_host=False)
        for path, variant in order:
            for anchor in ((0, 1) if path == 3 else (0,)):  # anchor 1: the sincos VALU kernel's own tiles
                ctx.set_option(capi.OPT_SYNTH_PATH, path)
                ctx.set_option(capi.OPT_VALU_VARIANT, variant)
                ctx.set_option(capi.OPT_ANCHOR, anchor)
                ctx.debug_fill_out(np.nan)
                got = ctx.batch_synth(1234, 0, 256)
                assert np.all(np.isfinite(got)), (path, variant, anchor)
                assert_parity(got, want, TOL)
    finally:
        ctx.set_options(shipped)


def test_batch_from_z_vs_oracle(ctx):
    rng = np.random.default_rng(11)
    offs, toas, nu, segs, *_ = _build(ctx, rng)
    R, nmax = 33, max(s.n_modes for s in segs)
    z = rng.standard_normal((R, len(segs), len(offs) - 1, nmax, 2))
    got = ctx.batch_synth_from_z(z)
    zo = {s: z[:, s, :, :segs[s].n_modes, :] for s in range(len(segs))}
    want = O.batch_synth(offs, toas, nu, segs, 0, 0, R, z_override=zo)
    assert_parity(got, want, TOL)


@pytest.mark.parametrize("path", [2, 3])
@pytest.mark.parametrize("anchor", [0, 1, 3, 8, 64])
def test_recurrence_anchor_accuracy(ctx, capi, path, anchor):
    """The fused kernels' phasor recurrence stays within tolerance for every re-anchor interval
    (0 = once per signal, the default), on 100-mode grids with a FLAT spectrum (every mode
    weighs equally) and real-MJD-like epochs (t ~ 5e9 s, phases up to ~2e4 rad)."""
    rng = np.random.default_rng(5)
    offs, toas, nu = random_layout(rng, 4, (100, 300), t_max=1.6e8)
    toas = toas + 4.5e9
    ctx.batch_set_toas(offs, toas, nu)
    f, _ = per_psr_signal(rng, offs, toas, 100)
    a = np.full_like(f, 1e-7)
    ctx.batch_add_signal(0, f, a, idx=2.0)
    ctx.set_option(capi.OPT_SYNTH_PATH, path)
    ctx.set_option(capi.OPT_ANCHOR, anchor)
    try:
        got = ctx.batch_synth(5, 0, 64)
    finally:
        ctx.set_option(capi.OPT_SYNTH_PATH, 0)
        ctx.set_option(capi.OPT_ANCHOR, 0)
    want = O.batch_synth(offs, toas, nu, [O.Segment(0, 2 * np.pi * f, a, 2.0)], 5, 0, 64)
    assert_parity(got, want, TOL)


@pytest.mark.parametrize("white,ecorr", [(True, False), (False, True), (True, True)])
def test_white_fused_matches_separate_pass(ctx, capi, white, ecorr):
    """The seeded kernel's white/ECORR epilogue and the separate k_white_pairs pass draw the same
    normals: the two agree to rounding (only the order of the final additions differs)."""
    rng = np.random.default_rng(31)
    _build(ctx, rng, P=5, white=white, ecorr=ecorr)
    try:
        ctx.set_option(capi.OPT_SYNTH_PATH, 3)
        fused = ctx.batch_synth(77, 9, 131)
        ctx.set_option(capi.OPT_FUSE_WHITE, 0)
        separate = ctx.batch_synth(77, 9, 131)
    finally:
        ctx.set_option(capi.OPT_FUSE_WHITE, 1)
        ctx.set_option(capi.OPT_SYNTH_PATH, 0)
    assert_parity(fused, separate, 1e-13)


def test_batch_split_invariance_bitwise(ctx):
    """Realization r is bit-identical whatever batch it is drawn in (multi-GPU sharding contract)."""
    rng = np.random.default_rng(8)
    _build(ctx, rng, P=6, white=True)
    full = ctx.batch_synth(2024, 0, 200)
    parts = np.concatenate([ctx.batch_synth(2024, r0, n) for r0, n in ((0, 64), (64, 100), (164, 36))])
    np.testing.assert_array_equal(full, parts)
    again = ctx.batch_synth(2024, 0, 200)
    np.testing.assert_array_equal(full, again)


@pytest.mark.parametrize("mix_mfma", [1, 0], ids=["mfma", "valu"])
@pytest.mark.parametrize("factor", ["cholesky", "svd", "rank3"])
def test_tiled_mix_vs_oracle(ctx, capi, factor, mix_mfma):
    """P >= 64 takes the GEMM mix: k_mix_mfma (default) or the register-tiled VALU k_mix_tiled
    (FPTA_OPT_MIX_MFMA 0), triangular when L is a Cholesky factor, over the leading nonzero columns only for the
    batch path's rank-3 factor of the singular dipole ORF, dense for numpy's full SVD factor; P = 150 is not a
    multiple of the 64-pulsar tile. Both against the oracle, and the two mixes' coefficients against each other."""
    ctx.set_option(capi.OPT_MIX_MFMA, mix_mfma)
    from fakepta_amd.batch import batch_factor
    rng = np.random.default_rng(21)
    P = 150
    offs, toas, nu = random_layout(rng, P, (5, 40))
    ctx.batch_set_toas(offs, toas, nu)
    f, amp, _, pos = common_signal(rng, offs, toas, 17)
    if factor == "cholesky":
        L = batch_factor(O.orf_hd(pos))
        assert np.allclose(L, np.tril(L))
    elif factor == "svd":
        L = O.mvn_factor(O.orf_monopole(pos))  # numpy's full factor: every column nonzero (rounding noise)
        assert not np.allclose(L, np.tril(L)) and np.all(np.any(L != 0, axis=0))
    else:
        L = batch_factor(O.orf_dipole(pos))
        assert np.all(L[:, 3:] == 0) and not np.allclose(L, np.tril(L))
    ctx.batch_add_signal(1, f, amp, idx=0.0, L=L)
    f2, a2 = per_psr_signal(rng, offs, toas, 5)
    ctx.batch_add_signal(0, f2, a2, idx=4.0)
    segs = [O.Segment(1, 2 * np.pi * f, amp, 0.0, L=L), O.Segment(0, 2 * np.pi * f2, a2, 4.0)]
    try:
        for real0, R in ((0, 130), (77, 5)):
            got = ctx.batch_synth(31, real0, R)
            want = O.batch_synth(offs, toas, nu, segs, 31, real0, R)
            assert_parity(got, want, TOL)
        _, co = ctx.batch_synth(31, 0, 130, coeffs=True)
        ctx.set_option(capi.OPT_MIX_MFMA, 1 - mix_mfma)
        _, co_other = ctx.batch_synth(31, 0, 130, coeffs=True)
        assert_parity(co, co_other, 1e-13)
    finally:
        ctx.set_option(capi.OPT_MIX_MFMA, 1)


def test_checksums_device(ctx):
    rng = np.random.default_rng(9)
    _build(ctx, rng, P=4, white=True)
    out = ctx.batch_synth(1, 0, 50)
    s = ctx.batch_checksums()
    np.testing.assert_allclose(s[:, 0], out.sum(1), rtol=1e-9, atol=1e-12 * np.abs(out).sum(1).max())
    np.testing.assert_allclose(s[:, 1], (out ** 2).sum(1), rtol=1e-12)


def test_errors_are_loud(ctx, capi):
    with pytest.raises(capi.FptaError):
        ctx.batch_set_toas(np.array([0, 5, 5]), np.zeros(5), np.ones(5))  # empty pulsar
    with pytest.raises(capi.FptaError):
        ctx.set_option(capi.OPT_SYNTH_PATH, 7)
    with pytest.raises(capi.FptaError):
        ctx.batch_add_signal(1, np.ones(3), np.ones(3))  # common without ORF factor


# ----------------------------------------------------------------------------- C2 at full size
def test_c2_full_size(ctx):
    """BASELINE configs[1] shape: 100 psr x 2000 TOAs, RN30 + DM100 + HD30, R = 1024 on device.
    Size-independent checks: 4 realizations re-synthesized by the oracle from the device's own
    coefficients; determinism; per-realization checksums."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=100, Tobs=10, ntoas=2000, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": 100, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    info = ctx.batch_info()
    assert info["n_toa"] == 200000 and info["K"] == 320
    out, co = sim.synth(1024, seed=1234, coeffs=True)
    # a coefficient download needs every coefficient in the coefficient buffer, so this block runs the two-kernel path
    # (k_gen draws, k_grid_dft_mfma, k_grid_interp_ws): the same draws; the shipped fused kernel is asserted on the
    # second synth below (bit-identical to this block on whole-chunk bands, to rounding on half-chunk bands) and by
    # test_c2_full_size_gridded_vs_seeded against the oracle
    assert ctx.batch_grid_info()["interp_kernel"] == "k_grid_interp_ws<false>", ctx.batch_grid_info()
    assert np.all(np.isfinite(out))
    pick = [0, 1, 511, 1023]
    segs = oracle_segments(sim)
    for r in pick:
        want = np.zeros(sim.n_toa)
        col = 0
        for s in segs:
            for p in range(len(psrs)):
                sl = slice(sim.offs[p], sim.offs[p + 1])
                w = s.w[p] if s.kind == 0 else s.w
                ph = np.outer(sim.toas[sl], w)
                ch = (s.freqf / sim.freqs[sl]) ** s.idx
                a = co[p, col:col + 2 * s.n_modes, r]
                want[sl] += ch * (np.cos(ph) @ a[0::2] + np.sin(ph) @ a[1::2])
            col += 2 * s.n_modes
        assert_parity(out[r], want, TOL)
    # coefficients follow the Philox stream of the oracle
    z = O.gp_normals(1234, np.array(pick), 17, 0, 30)
    want_c = sim.segments[0]["amp"][17][None, :] * z[:, :, 0]
    np.testing.assert_allclose(co[17, 0:60:2, pick], want_c, rtol=1e-13, atol=1e-14 * np.abs(want_c).max())
    s1 = sim.checksums()
    out2 = sim.synth(1024, seed=1234)
    kernel = ctx.batch_grid_info()["interp_kernel"]
    assert kernel.startswith("k_grid_fused<") and ", false, true, " in kernel, kernel  # draws in the kernel (GEN)
    if kernel.endswith(", false>"):  # whole-chunk bands: the two-kernel path's sums bit for bit
        np.testing.assert_array_equal(out, out2)
    else:
        assert rel_err(out2, out) <= 1e-12
    np.testing.assert_allclose(s1[:, 1], (out ** 2).sum(1), rtol=1e-12)
