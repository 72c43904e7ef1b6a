"""Statistical acceptance of the batched Philox path (the draws are not numpy's stream, so these
are the checks that the injected processes are the intended ones): PSD slope/amplitude recovery,
Hellings-Downs recovery, white/ECORR covariance. Run on an MI355X."""
import numpy as np
import pytest

from oracle import fakepta_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from fakepta_amd import _capi
    c = _capi.Context(0)
    yield c
    c.close()


def test_psd_slope_and_amplitude_recovered(ctx):
    """Least-squares Fourier projection of R realizations recovers psd_k * df_k per mode and the
    power-law slope (fake_pta.py:372-387 semantics: <a_k^2> = S(f_k) df_k)."""
    n, N, R = 600, 30, 4000
    T = 10 * O.JULIAN_YEAR
    toas = np.linspace(0, T, n)
    nu = np.full(n, 1400.0)
    f = O.freq_grid(N, T)
    log10_A, gamma = -13.5, 3.5
    psd = O.powerlaw(f, log10_A, gamma)
    df = O.delta_f(f)
    ctx.batch_set_toas(np.array([0, n]), toas, nu)
    ctx.batch_add_signal(0, f[None, :], np.sqrt(psd * df)[None, :], idx=0.0)
    out = ctx.batch_synth(77, 0, R)
    F = O.fourier_basis(toas, nu, f, 0.0)
    coef = np.linalg.lstsq(F, out.T, rcond=None)[0]  # [2N, R]
    var = 0.5 * ((coef[0::2] ** 2).mean(1) + (coef[1::2] ** 2).mean(1))
    ratio = var / (psd * df)
    tol = 5 * np.sqrt(1.0 / R)  # std of a variance estimate from 2R samples is sqrt(2/(2R))
    assert np.all(np.abs(ratio - 1) < tol), ratio
    slope = np.polyfit(np.log(f), np.log(var / df), 1)[0]
    assert abs(-slope - gamma) < 0.05
    amp = np.exp(np.mean(np.log(var / (df * O.powerlaw(f, 0.0, gamma)))))
    assert abs(0.5 * np.log10(amp) - log10_A) < 0.02


def test_hellings_downs_recovered(ctx):
    """Pairwise zero-lag correlations of the common process follow the HD curve
    (estimators of correlated_noises.py:14-47 on identical TOAs)."""
    P, n, N, R = 40, 200, 30, 1500
    i = np.arange(P) + 0.5
    cost = 1 - 2 * i / P
    phi = np.mod(2 * np.pi * i / ((1 + 5 ** 0.5) / 2), 2 * np.pi)
    th = np.arccos(cost)
    pos = np.stack([np.cos(phi) * np.sin(th), np.sin(phi) * np.sin(th), np.cos(th)], 1)
    T = 10 * O.JULIAN_YEAR
    toas = np.tile(np.linspace(0, T, n), P)
    offs = np.arange(P + 1) * n
    gam = O.orf_hd(pos)
    f = O.freq_grid(N, T)
    amp = np.sqrt(O.powerlaw(f, -14.0, 13 / 3) * O.delta_f(f))
    ctx.batch_set_toas(offs, toas, np.full(P * n, 1400.0))
    ctx.batch_add_signal(1, f, amp, idx=0.0, L=O.mvn_factor(gam))
    out, co = ctx.batch_synth(5, 0, R, coeffs=True)
    # coefficient level: x = L z has covariance Gamma
    x = co / amp.repeat(2)[None, :, None]  # [P, 2N, R]
    x = x.reshape(P, -1)
    cov = x @ x.T / x.shape[1]
    assert np.max(np.abs(cov - gam)) < 6 / np.sqrt(x.shape[1])
    # time domain: normalized zero-lag cross-correlation, binned in angle
    r = out.reshape(R, P, n)
    c = np.einsum("rpt,rqt->pq", r, r) / (R * n)
    rho = c / np.sqrt(np.outer(np.diag(c), np.diag(c)))
    iu = np.triu_indices(P, 1)
    ang = np.arccos(np.clip(pos @ pos.T, -1, 1))[iu]
    edges = np.linspace(0, np.pi, 8)
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (ang > lo) & (ang < hi)
        if sel.sum() < 10:
            continue
        assert abs(rho[iu][sel].mean() - gam[iu][sel].mean()) < 0.03


def test_device_correlations_match_numpy(ctx):
    """fpta_batch_correlations (all modes) == numpy on the same block (deterministic sums)."""
    rng = np.random.default_rng(4)
    P, n, R = 70, 150, 40
    offs = np.arange(P + 1) * n
    toas = np.tile(np.sort(rng.uniform(0, 3e8, n)), P)
    ctx.batch_set_toas(offs, toas, np.full(P * n, 1400.0))
    v = rng.normal(size=(P, 3))
    f = O.freq_grid(20, 3e8)
    ctx.batch_add_signal(1, f, np.sqrt(O.powerlaw(f, -14, 4.0) * O.delta_f(f)), L=O.mvn_factor(
        O.orf_hd(v / np.linalg.norm(v, axis=1)[:, None])))
    ctx.batch_set_white(np.full(P * n, 1e-7))
    out = ctx.batch_synth(8, 0, R).reshape(R, P, n)
    C = np.einsum("rat,rbt->rab", out, out) / n
    scale = np.abs(C).max()
    np.testing.assert_allclose(ctx.batch_correlations(0), C, rtol=1e-12, atol=1e-13 * scale)
    np.testing.assert_allclose(ctx.batch_correlations(1), C.sum(0), rtol=1e-12, atol=1e-13 * scale * R)
    d = np.sqrt(np.einsum("raa->ra", C))
    np.testing.assert_allclose(ctx.batch_correlations(3), d ** 2, rtol=1e-12)
    np.testing.assert_allclose(ctx.batch_correlations(2), (C / (d[:, :, None] * d[:, None, :])).sum(0),
                               rtol=1e-11, atol=1e-12 * R)
    np.testing.assert_array_equal(ctx.batch_correlations(2), ctx.batch_correlations(2))


def test_hd_curve_on_device():
    """BatchSimulator.hd_curve recovers Hellings-Downs from on-device statistics."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    np.random.seed(2)
    psrs = fp.make_fake_array(npsrs=50, Tobs=10, ntoas=300, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="X.1400", custom_model={"RN": None, "DM": None, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-14, gamma=13 / 3, components=30)
    sim = BatchSimulator(psrs, white=False)
    sim.synth(2048, seed=11, to_host=False)
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # empty bins must not warn
        mean, std, centres, counts = sim.hd_curve(bins=40, return_counts=True)
    assert np.array_equal(np.isnan(mean), counts == 0) and counts.sum() == 50 * 49 // 2
    mean, std, centres = sim.hd_curve(bins=8)
    pos = np.array([p.pos for p in psrs])
    gam = O.orf_hd(pos)
    iu = np.triu_indices(len(psrs), 1)
    ang = np.arccos(np.clip(pos @ pos.T, -1, 1))[iu]
    edges = np.linspace(0, np.pi, 9)
    for k in range(8):
        sel = (ang > edges[k]) & (ang < edges[k + 1])
        if sel.sum() >= 5:
            assert abs(mean[k] - gam[iu][sel].mean()) < 0.03


def test_white_and_ecorr_covariance(ctx):
    n, R = 400, 20000
    rng = np.random.default_rng(1)
    sigma = rng.uniform(1e-7, 1e-6, n)
    blocks = [np.arange(s, s + 4) for s in range(0, n, 4)]
    es = np.full(len(blocks), 5e-7)
    ctx.batch_set_toas(np.array([0, n]), np.linspace(0, 3e8, n), np.full(n, 1400.0))
    ctx.batch_set_white(sigma, blocks, es)
    out = ctx.batch_synth(3, 0, R)
    var = out.var(0)
    np.testing.assert_allclose(var, sigma ** 2 + es[0] ** 2, rtol=6 * np.sqrt(2 / R))
    inblock = np.mean(out[:, 0] * out[:, 1])
    across = np.mean(out[:, 3] * out[:, 4])
    assert abs(inblock / es[0] ** 2 - 1) < 0.1
    assert abs(across) < 0.05 * es[0] ** 2 + 5 * np.sqrt(var[3] * var[4] / R)
