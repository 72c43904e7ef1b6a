"""Pin the CPU oracle (oracle/fakepta_oracle.py) against the reference's own outputs
(tests/golden/, generated from /root/reference by tools/gen_golden.py). CPU only."""
import json

import numpy as np
import pytest

from oracle import fakepta_oracle as O
from tests.conftest import assert_parity


def test_psd_all_six(golden):
    g = golden("g1_psd.npz")
    meta = json.loads(str(g["meta_json"]))
    n = 0
    for key, params in meta.items():
        name, gi, _ = key.split("__")
        f = g["grid" + gi[1:]]
        p = {k: (np.array(v) if isinstance(v, list) else v) for k, v in params.items()}
        out = O.PSDS[name](f.copy(), **p)
        np.testing.assert_allclose(out, g[key], rtol=1e-13, atol=0)
        n += 1
    assert n == 6 * 9


def test_tutorial_psd_known_answer(golden):
    ka = golden("g5_tutorial.json")
    T = 1.0 / ka["rn_f_first"]
    f = O.freq_grid(30, T)
    psd = O.powerlaw(f, -14.0, 3)
    np.testing.assert_allclose(psd, ka["rn_psd_log10A_m14_gamma3_30modes_Tobs10"], rtol=1e-8)


@pytest.mark.parametrize("lab", ["rn", "dm", "sv"])
def test_single_pulsar_gp(golden, lab):
    g = golden("g2_single_psr.npz")
    toas, freqs = g["toas"], g["freqs"]
    f, psd, z, idx = g[f"{lab}_f"], g[f"{lab}_psd"], g[f"{lab}_z"], g[f"{lab}_idx"]
    np.testing.assert_allclose(f, O.freq_grid(len(f), float(g["Tspan"])), rtol=0, atol=0)
    coeffs = O.gp_coeffs_from_z(psd, z)
    np.testing.assert_allclose(O.gp_fourier(coeffs, f), g[f"{lab}_fourier"], rtol=1e-15)
    # loop-faithful restatement reproduces the injected residual increment
    delta = O.gp_synth_loop(toas, freqs, f, coeffs, idx)
    assert_parity(delta, g[f"{lab}_delta"], 1e-13)
    # vectorised form
    df = O.delta_f(f)
    vec = O.gp_synth_vec(toas, freqs, f, df ** 0.5 * coeffs[0::2], df ** 0.5 * coeffs[1::2], idx)
    assert_parity(vec, g[f"{lab}_delta"], 1e-12)
    # reconstruct_signal
    rec = O.reconstruct_loop(toas, freqs, f, g[f"{lab}_fourier"], idx)
    assert_parity(rec, g[f"{lab}_reconstruct"], 1e-13)


def test_reinject_replaces(golden):
    g = golden("g2_single_psr.npz")
    toas, freqs = g["toas"], g["freqs"]
    old = O.reconstruct_loop(toas, freqs, g["rn_f"], g["rn_fourier"], 0.0)
    coeffs = O.gp_coeffs_from_z(g["rn2_psd"], g["rn2_z"])
    new = O.gp_synth_loop(toas, freqs, g["rn_f"], coeffs, 0.0)
    assert_parity(g["rn2_before"] - old + new, g["rn2_residuals"], 1e-12)


def test_white_noise(golden):
    g = golden("g2_single_psr.npz")
    flags = g["backend_flags"]
    efac = dict(zip(["A.1400", "B.800"], g["wn_efac"]))
    eq = dict(zip(["A.1400", "B.800"], g["wn_tnequad"]))
    sig = O.white_sigma(g["toaerrs"], flags, efac, eq)
    # wn_delta = after - before carries the cancellation error of the GP residual it sits on
    assert_parity(sig * g["wn_z"], g["wn_delta"], 1e-11)


def test_quantise_ecorr_preserves_d2(golden):
    g = golden("g2_single_psr.npz")
    flags = g["q_flags"]
    q = O.quantise_ecorr(g["q_toas"], flags, np.unique(flags))
    assert [len(b) for b in q] == list(g["q_lens"])
    np.testing.assert_array_equal(np.concatenate(q), g["q_idx"])
    fixed = O.ecorr_blocks(g["q_toas"], flags, np.unique(flags))
    assert len(fixed) == len(q) + len(np.unique(flags))
    assert sorted(np.concatenate(fixed).tolist()) == list(range(len(g["q_toas"])))


@pytest.mark.parametrize("orf", ["hd", "monopole", "dipole", "curn"])
def test_common_correlated(golden, orf):
    g = golden("g3_common.npz")
    offs, toas, freqs, pos = g["offs"], g["toas"], g["freqs"], g["pos"]
    gam = O.ORFS[orf](pos)
    np.testing.assert_allclose(gam, g[f"{orf}_orf"], rtol=1e-14, atol=1e-15)
    L = O.mvn_factor(gam)
    np.testing.assert_allclose(L.T, g[f"{orf}_svdM"], rtol=0, atol=1e-13)
    P = len(offs) - 1
    tl = [toas[offs[i]:offs[i + 1]] for i in range(P)]
    fl = [freqs[offs[i]:offs[i + 1]] for i in range(P)]
    res, fourier = O.common_synth_loop(tl, fl, g[f"{orf}_f"], g[f"{orf}_psd"], g[f"{orf}_z"],
                                       g[f"{orf}_svdM"].T, g[f"{orf}_idx"])
    np.testing.assert_allclose(fourier, g[f"{orf}_fourier"], rtol=1e-12, atol=1e-12 * np.abs(fourier).max())
    assert_parity(np.concatenate(res), g[f"{orf}_residuals"], 1e-12)
    # reconstruct from the stored coefficients
    rec = np.concatenate([O.reconstruct_loop(tl[i], fl[i], g[f"{orf}_f"], g[f"{orf}_fourier"][i], g[f"{orf}_idx"])
                          for i in range(P)])
    assert_parity(rec, g[f"{orf}_reconstruct"], 1e-12)


def test_common_components_not_len_f_g9(golden):
    """components != len(f_psd) (correlated_noises.py:140-160): 30 modes of a 40-frequency grid are injected and
    stored with the full f / psd; with 20 frequencies the loop fails at mode 20 (IndexError), as in fixture G9."""
    g = golden("g9_common_components.npz")
    offs, toas, freqs = g["offs"], g["toas"], g["freqs"]
    P = len(offs) - 1
    tl = [toas[offs[i]:offs[i + 1]] for i in range(P)]
    fl = [freqs[offs[i]:offs[i + 1]] for i in range(P)]
    L = O.mvn_factor(O.orf_hd(g["pos"]))
    assert len(g["long_f"]) == 40 and len(g["long_psd"]) == 40 and int(g["long_nbin"]) == 30
    res, fourier = O.common_synth_loop(tl, fl, g["long_f"], g["long_psd"], g["long_z"], L, 2.0, components=30)
    np.testing.assert_allclose(fourier, g["long_fourier"], rtol=1e-12, atol=1e-12 * np.abs(fourier).max())
    assert_parity(np.concatenate(res), g["long_residuals"], 1e-12)
    rec = np.concatenate([O.reconstruct_loop(tl[i], fl[i], g["long_f"][:30], g["long_fourier"][i], 2.0)
                          for i in range(P)])
    assert_parity(rec, g["long_reconstruct"], 1e-12)
    f20 = g["long_f"][:20]
    with pytest.raises(IndexError, match=str(g["short_error"])):
        O.common_synth_loop(tl, fl, f20, O.powerlaw(f20, -14.5, 13 / 3), g["short_z"], L, 0.0, components=30)


def test_philox_known_answers():
    kat = [((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
           ((0xffffffff,) * 4, (0xffffffff,) * 2, (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
           ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
            (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1))]
    for c, k, exp in kat:
        out = O.philox4x32_10(np.array([c], np.uint32), np.array(k, np.uint32))
        assert tuple(int(x) for x in out[0]) == exp


def test_box_muller_moments():
    z = O.gp_normals(1234, np.arange(4000), 3, 1, 50).ravel()
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    w = O.white_normals(99, np.arange(10), 20001)
    assert abs(w.mean()) < 0.01 and abs(w.std() - 1) < 0.01


def test_normal_map_accuracy_and_moments():
    """The build's uniform -> normal map (oracle.normals4, restated on the device by philox.h normals4): its fp64
    polynomial log and sine / cosine agree with numpy's to 5e-14 over 2e6 random words and the end points, and
    four normals per Philox call have the standard normal's moments and tails (|z| <= sqrt(64 ln 2))."""
    a = np.random.default_rng(0).integers(0, 2 ** 32, size=2_000_000, dtype=np.uint64).astype(np.uint32)
    a[:3] = [0, 0xFFFFFFFF, 1]
    ref = np.log((a.astype(np.float64) + 1.0) * 2.0 ** -32)
    got = O.bm_log_u32(a)
    assert got[1] == 0.0 and np.max(np.abs(got - ref)) <= 5e-14 * np.max(np.abs(ref))
    nz = ref != 0
    assert np.max(np.abs(got[nz] - ref[nz]) / np.abs(ref[nz])) <= 5e-14
    u = a.astype(np.float64) * 2.0 ** -32
    sn, cs = O.bm_sincos2pi_u32(a)
    assert np.max(np.abs(sn - np.sin(2 * np.pi * u))) <= 5e-14 and np.max(np.abs(cs - np.cos(2 * np.pi * u))) <= 5e-14
    ctr = np.stack([np.arange(400_000, dtype=np.uint32), np.full(400_000, 7, np.uint32),
                    np.full(400_000, 3, np.uint32), np.arange(400_000, dtype=np.uint32) // 3], -1)
    z = O.normals4(O.philox4x32_10(ctr, np.array([11, 12], np.uint32)))
    assert z.shape == (400_000, 4)
    flat = z.ravel()
    assert abs(flat.mean()) < 5e-3 and abs(flat.std() - 1) < 5e-3
    assert abs(np.mean(flat ** 4) - 3.0) < 0.03 and np.max(np.abs(flat)) <= np.sqrt(64 * np.log(2)) + 1e-12
    assert abs(np.mean(np.abs(flat) > 3) - 2.6998e-3) < 3e-4
    c = np.corrcoef(z.T)
    assert np.max(np.abs(c - np.eye(4))) < 5e-3


def test_batch_semantics_match_reference_loop():
    """The batch layout (per-pulsar + common segment, explicit z) reproduces the loop-faithful
    reference restatements on the same draws."""
    rng = np.random.default_rng(0)
    P, N = 4, 6
    offs = np.array([0, 30, 55, 90, 120])
    toas = np.concatenate([np.sort(rng.uniform(0, 3e8, offs[i + 1] - offs[i])) for i in range(P)])
    freqs = rng.normal(1400, 10, offs[-1])
    T = [np.ptp(toas[offs[i]:offs[i + 1]]) for i in range(P)]
    f_p = np.array([O.freq_grid(N, t) for t in T])
    psd_p = np.array([O.powerlaw(f, -13.5, 3.0) for f in f_p])
    amp_p = np.sqrt(psd_p * np.array([O.delta_f(f) for f in f_p]))
    fc = O.freq_grid(N, toas.max() - toas.min())
    psdc = O.powerlaw(fc, -14.0, 13 / 3)
    v = rng.normal(size=(P, 3))
    L = O.mvn_factor(O.orf_hd(v / np.linalg.norm(v, axis=1)[:, None]))
    segs = [O.Segment(0, 2 * np.pi * f_p, amp_p, idx=2.0),
            O.Segment(1, 2 * np.pi * fc, np.sqrt(psdc * O.delta_f(fc)), idx=0.0, L=L)]
    z0 = rng.standard_normal((1, P, N, 2))
    z1 = rng.standard_normal((1, P, N, 2))
    out = O.batch_synth(offs, toas, freqs, segs, 0, 0, 1, z_override={0: z0, 1: z1})[0]
    ref = np.zeros(offs[-1])
    for p in range(P):
        sl = slice(offs[p], offs[p + 1])
        c = np.empty(2 * N)
        c[0::2] = np.sqrt(psd_p[p]) * z0[0, p, :, 0]
        c[1::2] = np.sqrt(psd_p[p]) * z0[0, p, :, 1]
        ref[sl] += O.gp_synth_loop(toas[sl], freqs[sl], f_p[p], c, 2.0)
    zc = np.stack([z1[0, :, :, 1].T, z1[0, :, :, 0].T], axis=1)  # [N, 2(sin, cos), P]
    res, _ = O.common_synth_loop([toas[offs[i]:offs[i + 1]] for i in range(P)],
                                 [freqs[offs[i]:offs[i + 1]] for i in range(P)], fc, psdc, zc, L, 0.0)
    ref += np.concatenate(res)
    assert_parity(out, ref, 1e-12)


def test_dense_covariance_oracle_vs_g6(golden):
    """make_time_correlated_noise_cov / make_noise_covariance_matrix / draw_noise_model(residuals)
    restated in oracle.dense_* reproduce the reference's outputs (fake_pta.py:389-420, :493-524)."""
    g = golden("g6_dense_cov.npz")
    sigs = []
    for lab in ("rn", "dm", "sv"):
        f, psd, idx = g[f"{lab}_f"], g[f"{lab}_psd"], float(g[f"{lab}_idx"])
        assert_parity(O.dense_cov_signal(g["toas"], g["freqs"], f, psd, idx), g[f"{lab}_cov"], 1e-14)
        sigs.append((f, psd, idx))
    red = O.dense_cov(g["toas"], g["freqs"], sigs)
    assert_parity(red, g["red_cov"], 1e-14)
    flags = g["backend_flags"]
    sig = np.zeros(len(g["toas"]))
    for b, ef, tq in zip(("A.1400", "B.800"), g["efac"], g["tnequad"]):
        m = flags == b
        sig[m] = np.sqrt(ef ** 2 * g["toaerrs"][m] ** 2 + 10 ** (2 * tq))
    assert_parity(sig ** 2, g["white_cov"], 1e-15)
    assert_parity(O.wiener_reference(g["white_cov"], red, g["residuals"]), g["wiener"], 1e-12)


def test_dense_draws_oracle_distribution():
    """dense_draws = cholesky(C) z with the DENSE_STREAM normals: x x^T / R -> C."""
    rng = np.random.default_rng(1)
    A = rng.normal(size=(6, 6))
    C = A @ A.T + 6 * np.eye(6)
    x = O.dense_draws(C, 5, 0, 40000)
    S = x.T @ x / len(x)
    assert np.max(np.abs(S - C) / np.sqrt(np.outer(np.diag(C), np.diag(C)))) < 0.03


# ----------------------------------------------------------------------------- gridded-path model
@pytest.mark.parametrize("n_modes,spectrum", [(30, "flat"), (100, "flat"), (100, "red"), (7, "flat")])
def test_grid_model_error_bound(n_modes, spectrum):
    """The gridded factorisation (grid.hip) at its defaults (width 13, oversampling 2) reproduces the
    direct sum to <= 2e-11 relative on real-MJD-like epochs, flat spectrum being the worst case."""
    rng = np.random.default_rng(n_modes)
    T = 3.15e8
    toas = np.sort(rng.uniform(0, T, 1500)) + 4.8e9
    freqs = rng.uniform(700, 3000, toas.size)
    f = np.arange(1, n_modes + 1) / T
    amp = np.ones(n_modes) if spectrum == "flat" else np.arange(1, n_modes + 1) ** (-13 / 6)
    c = rng.normal(size=(3, n_modes)) * amp
    s = rng.normal(size=(3, n_modes)) * amp
    want = O.gp_synth_vec(toas, freqs, f, c, s, 2.0)
    got = O.grid_synth(toas, freqs, 2 * np.pi * f[0], c, s, 2.0)
    err = np.linalg.norm(got - want) / np.linalg.norm(want)
    assert err <= 2e-11, err
    coarse = O.grid_synth(toas, freqs, 2 * np.pi * f[0], c, s, 2.0, w=6)
    assert np.linalg.norm(coarse - want) / np.linalg.norm(want) > 1e-9  # the width controls the error
