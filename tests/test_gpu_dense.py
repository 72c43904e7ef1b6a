"""Dense-covariance path on the GPU through the C-ABI, against the
reference's golden vectors (tests/golden/g6_dense_cov.npz) and the oracle.

Tolerances: covariances <= 1e-10 (fp64, as §8(c)); the Wiener estimate <= 1e-10 on the fixture
(condition number 1.6e3); Cholesky draws <= 1e-9 against numpy's Cholesky of the same matrix with
the same normals (both factors are backward stable; condition numbers below 1e5 here)."""
import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def capi():
    from fakepta_amd import _capi
    return _capi


@pytest.fixture(scope="module")
def ctx(capi):
    c = capi.Context(0)
    yield c
    c.close()


def _segs(g, labs=("rn", "dm", "sv")):
    return [(g[f"{lab}_f"], g[f"{lab}_psd"] * O.delta_f(g[f"{lab}_f"]), float(g[f"{lab}_idx"]), 1400.0)
            for lab in labs]


@pytest.mark.parametrize("lab", ["rn", "dm", "sv"])
def test_covariance_per_signal_vs_reference(ctx, golden, lab):
    g = golden("g6_dense_cov.npz")
    cov = ctx.gp_covariance(g["toas"], g["freqs"], _segs(g, (lab,)))
    assert_parity(cov, g[f"{lab}_cov"], 1e-10)
    np.testing.assert_array_equal(cov, cov.T)


def test_noise_covariance_and_wiener_vs_reference(ctx, golden):
    g = golden("g6_dense_cov.npz")
    red = ctx.gp_covariance(g["toas"], g["freqs"], _segs(g))
    assert_parity(red, g["red_cov"], 1e-10)
    tot = ctx.gp_covariance(g["toas"], g["freqs"], _segs(g), white_var=g["white_cov"])
    assert_parity(tot, g["red_cov"] + np.diag(g["white_cov"]), 1e-10)
    w = ctx.noise_wiener(g["toas"], g["freqs"], _segs(g), g["white_cov"], g["residuals"])
    assert_parity(w, g["wiener"], 1e-10)


def test_dropin_pulsar_covariance_replay(golden):
    """The reference's call sequence of tools/gen_golden.py gen_g6 through fakepta.fake_pta.Pulsar."""
    from fakepta import fake_pta as fp
    g = golden("g6_dense_cov.npz")
    rng = np.random.default_rng(17)
    yr = 365.25 * 24 * 3600
    keep = rng.random(80) < 0.75
    epochs = 0.2 * yr + np.arange(1, 81)[keep] * (30.1 * 24 * 3600)
    np.random.seed(23)
    psr = fp.Pulsar(epochs, 2e-7, 0.4, 2.2, pdist=(1.0, 0.2), freqs=[1400], backends=["A.1400", "B.800"],
                    custom_model={"RN": 30, "DM": 100, "Sv": 30})
    np.testing.assert_array_equal(psr.toas, g["toas"])
    for b in psr.backends:
        psr.noisedict[f"{psr.name}_{b}_efac"] = {"A.1400": 1.2, "B.800": 0.9}[b]
        psr.noisedict[f"{psr.name}_{b}_log10_tnequad"] = {"A.1400": -6.8, "B.800": -7.1}[b]
    psr.add_red_noise(spectrum="powerlaw", log10_A=-13.9, gamma=3.1)
    psr.add_dm_noise(spectrum="powerlaw", log10_A=-13.5, gamma=2.2)
    psr.add_chromatic_noise(spectrum="powerlaw", log10_A=-13.8, gamma=1.8)
    psr.add_white_noise()
    assert_parity(psr.residuals, g["residuals"], 1e-10)
    for sig, lab in (("red_noise", "rn"), ("dm_gp", "dm"), ("chrom_gp", "sv")):
        assert_parity(psr.make_time_correlated_noise_cov(signal=sig), g[f"{lab}_cov"], 1e-10)
    white_cov, red_cov = psr.make_noise_covariance_matrix()
    assert_parity(white_cov, g["white_cov"], 1e-14)
    assert_parity(red_cov, g["red_cov"], 1e-10)
    assert_parity(psr.draw_noise_model(residuals=g["residuals"]), g["wiener"], 1e-10)
    d = psr.draw_noise_model()
    assert d.shape == psr.toas.shape and np.all(np.isfinite(d))


def _random_case(seed, n, modes=((30, 0.0), (100, 2.0), (30, 4.0)), white_scale=3e-7):
    rng = np.random.default_rng(seed)
    yr = 365.25 * 86400
    toas = np.sort(rng.uniform(0.0, 12 * yr, n)) + 53000 * 86400.0
    nu = rng.choice([800.0, 1400.0, 2100.0], n) + rng.normal(0, 5, n)
    T = max(toas.max() - toas.min(), yr)
    segs, osigs = [], []
    for nm, idx in modes:
        f = np.arange(1, nm + 1) / T
        psd = O.powerlaw(f, rng.uniform(-14.5, -13.5), rng.uniform(1.5, 4.5))
        segs.append((f, psd * O.delta_f(f), idx, 1400.0))
        osigs.append((f, psd, idx))
    white = (white_scale * rng.uniform(0.5, 2.0, n)) ** 2
    return toas, nu, segs, osigs, white


@pytest.mark.parametrize("n", [1, 63, 64, 65, 777, 2000])
def test_covariance_vs_oracle_sizes(ctx, n):
    toas, nu, segs, osigs, white = _random_case(n, n)
    got = ctx.gp_covariance(toas, nu, segs, white_var=white)
    want = O.dense_cov(toas, nu, osigs) + np.diag(white)
    assert_parity(got, want, 1e-10)


@pytest.mark.parametrize("n", [5, 64, 300, 777, 1500])
def test_wiener_vs_oracle_sizes(ctx, n):
    """Multi-panel Cholesky (n > 64, ragged last panel) + both substitutions."""
    toas, nu, segs, osigs, white = _random_case(100 + n, n)
    red = O.dense_cov(toas, nu, osigs)
    r = np.random.default_rng(n).multivariate_normal(np.zeros(n), red + np.diag(white))
    got = ctx.noise_wiener(toas, nu, segs, white, r)
    cov = red + np.diag(white)
    cond = np.linalg.cond(cov)
    want = red @ np.linalg.solve(cov, r)
    assert_parity(got, want, max(1e-10, 1e-15 * cond))
    assert_parity(got, O.wiener_reference(white, red, r), max(1e-10, 1e-15 * cond))


@pytest.mark.parametrize("n", [64, 333, 1000])
def test_draws_vs_oracle_and_split_invariance(ctx, n):
    toas, nu, segs, osigs, white = _random_case(200 + n, n, white_scale=1e-6)
    cov = O.dense_cov(toas, nu, osigs) + np.diag(white)
    got = ctx.noise_draw(toas, nu, segs, white, 4242, 7, 37)
    want = O.dense_draws(cov, 4242, 7, 37)
    assert_parity(got, want, 1e-9)
    part = ctx.noise_draw(toas, nu, segs, white, 4242, 20, 9)
    np.testing.assert_array_equal(part, got[13:22])


def test_draws_statistics(ctx):
    """Sample covariance of 20000 draws matches C (|S - C|_ij <= 6 sqrt((C_ii C_jj + C_ij^2) / R))."""
    toas, nu, segs, osigs, white = _random_case(9, 40, modes=((10, 0.0),), white_scale=1e-6)
    cov = O.dense_cov(toas, nu, osigs) + np.diag(white)
    R = 20000
    x = ctx.noise_draw(toas, nu, segs, white, 99, 0, R)
    S = x.T @ x / R
    d = np.sqrt(np.diag(cov))
    bound = 6 * np.sqrt((np.outer(d, d) ** 2 + cov ** 2) / R)
    assert np.all(np.abs(S - cov) <= bound)


def test_not_positive_definite_is_loud(ctx, capi):
    toas, nu, segs, _, _ = _random_case(3, 300, modes=((5, 0.0),))
    with pytest.raises(capi.FptaError, match="positive definite"):
        ctx.noise_draw(toas, nu, segs, np.zeros(300), 1, 0, 4)
    with pytest.raises(capi.FptaError):
        ctx.gp_covariance(toas, nu, [(segs[0][0], -segs[0][1], 0.0, 1400.0)])
