"""CPU ORACLE for the Fourier-basis GP residual synthesis path — TEST INFRASTRUCTURE ONLY.

This module is a plain numpy restatement of the reference algorithm
(mfalxa/fakepta @ 2025-08-08, /root/reference), used as the CHECKER for the HIP
product path. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import it. The product packages (fakepta, fakepta_amd) never import it and has
no CPU fallback.

Parity pinning: every reference-semantics function below is checked against the
committed golden vectors in tests/golden/ (generated in the build container by
tools/gen_golden.py, which imports the real reference) — see
tests/test_oracle_golden.py. The batch semantics (Philox draws, ORF mixing
order, white/ECORR streams) are new in this build and are specified here; the
Philox core is pinned by the Random123 known-answer vectors.

Two restatements of the synthesis are provided:
  * loop-faithful  — same per-mode elementwise structure as fake_pta.py:385-387
                     and correlated_noises.py:153-160 (used for the CPU baseline)
  * vectorised     — basis F (n_toa x 2N) times coefficients (used for checking
                     larger cases quickly)
"""
import numpy as np

# fakepta/constants.py:23-25 (copy of enterprise.constants): yr = Julian year, fyr = 1/yr
JULIAN_YEAR = 365.25 * 86400.0
FYR = 1.0 / JULIAN_YEAR
TWO_PI = 2.0 * np.pi


# ----------------------------------------------------------------------------- PSDs
# fakepta/spectrum.py:12-86 (ENTERPRISE gp_priors forms)

def powerlaw(f, log10_A, gamma):
    """fakepta/spectrum.py:12-15"""
    return (10 ** log10_A) ** 2 / (12.0 * np.pi ** 2) * FYR ** (gamma - 3) * f ** (-gamma)


def turnover(f, log10_A=-15, gamma=4.33, lf0=-8.5, kappa=10 / 3, beta=0.5):
    """fakepta/spectrum.py:18-20"""
    hcf = 10 ** log10_A * (f / FYR) ** ((3 - gamma) / 2) / (1 + (10 ** lf0 / f) ** kappa) ** beta
    return hcf ** 2 / 12 / np.pi ** 2 / f ** 3


def t_process(f, log10_A=-15, gamma=4.33, alphas=None):
    """fakepta/spectrum.py:23-29"""
    alphas = np.ones_like(f) if alphas is None else alphas
    return powerlaw(f, log10_A=log10_A, gamma=gamma) * alphas


def t_process_adapt(f, log10_A=-15, gamma=4.33, alphas_adapt=None, nfreq=None):
    """fakepta/spectrum.py:32-46"""
    if alphas_adapt is None:
        alpha_model = np.ones_like(f)
    elif nfreq is None:
        alpha_model = alphas_adapt
    else:
        alpha_model = np.ones_like(f)
        alpha_model[int(np.rint(nfreq))] = alphas_adapt
    return powerlaw(f, log10_A=log10_A, gamma=gamma) * alpha_model


def turnover_knee(f, log10_A, gamma, lfb, lfk, kappa, delta):
    """fakepta/spectrum.py:49-66"""
    hcf = (10 ** log10_A * (f / FYR) ** ((3 - gamma) / 2) * (1.0 + (f / 10 ** lfk)) ** delta
           / np.sqrt(1 + (10 ** lfb / f) ** kappa))
    return hcf ** 2 / 12 / np.pi ** 2 / f ** 3


def broken_powerlaw(f, log10_A, gamma, delta, log10_fb, kappa=0.1):
    """fakepta/spectrum.py:69-86"""
    hcf = (10 ** log10_A * (f / FYR) ** ((3 - gamma) / 2)
           * (1 + (f / 10 ** log10_fb) ** (1 / kappa)) ** (kappa * (gamma - delta) / 2))
    return hcf ** 2 / 12 / np.pi ** 2 / f ** 3


PSDS = dict(powerlaw=powerlaw, turnover=turnover, t_process=t_process,
            t_process_adapt=t_process_adapt, turnover_knee=turnover_knee,
            broken_powerlaw=broken_powerlaw)


# ----------------------------------------------------------------------------- grids

def freq_grid(n_modes, tspan):
    """fakepta/fake_pta.py:264 (per pulsar) / correlated_noises.py:120 (global span)"""
    return np.arange(1, n_modes + 1) / tspan


def delta_f(f):
    """fakepta/fake_pta.py:370: df = diff([0, f]), so df_0 = f_0"""
    return np.diff(np.append(0.0, f))


def chromatic(freqs, idx, freqf=1400.0):
    """fakepta/fake_pta.py:386: (freqf / nu)**idx (code, not the tutorial's prose, is authoritative)"""
    return (freqf / freqs) ** idx


# ----------------------------------------------------------------------------- per-pulsar GP

def gp_coeffs_from_z(psd, z):
    """fakepta/fake_pta.py:372-374: coeffs = normal(0, sqrt(repeat(psd, 2))) == sqrt(psd_rep) * z"""
    return 0.0 + np.sqrt(np.repeat(psd, 2)) * z


def gp_fourier(coeffs, f):
    """fakepta/fake_pta.py:381: fourier = (c_even, c_odd) / sqrt(df)"""
    df = delta_f(f)
    return np.vstack((coeffs[::2] / df ** 0.5, coeffs[1::2] / df ** 0.5))


def gp_synth_loop(toas, freqs, f, coeffs, idx, freqf=1400.0, mask=None, residuals=None):
    """Loop-faithful restatement of fakepta/fake_pta.py:385-387 (in-place accumulate).

    mask: the reference applies `mask` to toas but not to the chromatic factor
    (defect D9: it raises for a partial mask); here the chromatic factor is masked too.
    """
    r = np.zeros(len(toas)) if residuals is None else residuals
    if mask is None:
        mask = np.ones(len(toas), dtype=bool)
    df = delta_f(f)
    chrom = (freqf / freqs[mask]) ** idx
    for i in range(len(f)):
        r[mask] += chrom * df[i] ** 0.5 * coeffs[2 * i] * np.cos(2 * np.pi * f[i] * toas[mask])
        r[mask] += chrom * df[i] ** 0.5 * coeffs[2 * i + 1] * np.sin(2 * np.pi * f[i] * toas[mask])
    return r


def fourier_basis(toas, freqs, f, idx, freqf=1400.0):
    """F[t, 2k] = chrom cos(2 pi f_k t), F[t, 2k+1] = chrom sin(...) — fake_pta.py:415-418 layout"""
    ph = np.outer(toas, TWO_PI * np.asarray(f))
    F = np.empty((len(toas), 2 * len(f)))
    ch = chromatic(freqs, idx, freqf)[:, None]
    F[:, 0::2] = ch * np.cos(ph)
    F[:, 1::2] = ch * np.sin(ph)
    return F


def gp_synth_vec(toas, freqs, f, amp_cos, amp_sin, idx, freqf=1400.0):
    """Vectorised: sum_k chrom (amp_cos_k cos + amp_sin_k sin); amp = sqrt(df) * coeff (inject)
    or df * fourier (reconstruct). Supports amp of shape [N] or [R, N] (returns [R, n_toa])."""
    F = fourier_basis(toas, freqs, f, idx, freqf)
    amp_cos = np.asarray(amp_cos)
    A = np.empty(amp_cos.shape[:-1] + (2 * amp_cos.shape[-1],))
    A[..., 0::2] = amp_cos
    A[..., 1::2] = amp_sin
    return A @ F.T


def reconstruct_loop(toas, freqs, f, fourier, idx, freqf=1400.0):
    """fakepta/fake_pta.py:538-545 (GP branch of reconstruct_signal)"""
    sig = np.zeros(len(toas))
    df = delta_f(f)
    for c_k, f_k, df_k in zip(fourier.T, f, df):
        sig += df_k * c_k[0] * (freqf / freqs) ** idx * np.cos(2 * np.pi * f_k * toas)
        sig += df_k * c_k[1] * (freqf / freqs) ** idx * np.sin(2 * np.pi * f_k * toas)
    return sig


# ----------------------------------------------------------------------------- ORFs

def orf_hd(pos):
    """fakepta/correlated_noises.py:62-71 (vectorised; NaN for coincident pulsars, defect D8)"""
    pos = np.asarray(pos)
    with np.errstate(divide="ignore", invalid="ignore"):
        omc2 = (1 - pos @ pos.T) / 2
        g = 1.5 * omc2 * np.log(omc2) - 0.25 * omc2 + 0.5
    np.fill_diagonal(g, 1.0)
    return g


def orf_monopole(pos):
    """fakepta/correlated_noises.py:91-93"""
    n = len(pos)
    return np.ones((n, n))


def orf_dipole(pos):
    """fakepta/correlated_noises.py:95-104"""
    pos = np.asarray(pos)
    g = pos @ pos.T
    np.fill_diagonal(g, 1.0)
    return g


def orf_curn(pos):
    """fakepta/correlated_noises.py:106-108"""
    return np.eye(len(pos))


ORFS = dict(hd=orf_hd, monopole=orf_monopole, dipole=orf_dipole, curn=orf_curn)


def mvn_factor(cov):
    """numpy legacy multivariate_normal (method='svd'), as called at correlated_noises.py:154-155:
    x = z @ (sqrt(s)[:, None] * vt). Returned as L = M.T so that x = L @ z."""
    _, s, vt = np.linalg.svd(cov)
    return (np.sqrt(s)[:, None] * vt).T


def common_synth_loop(toas_list, freqs_list, f, psd, z, L, idx, freqf=1400.0, components=None):
    """Loop-faithful restatement of fakepta/correlated_noises.py:140-160.

    z: [N, 2, P] standard normals in the reference's draw order (sin vector first, then cos).
    components: modes looped (default len(f)); fourier is [P, 2, components] (:142) and the loop runs over the
    first `components` entries of f, so components > len(f) raises IndexError as the reference does at :157.
    Returns (residual list, fourier [P, 2, components])."""
    P = len(toas_list)
    components = len(f) if components is None else int(components)
    df = delta_f(f)
    coeffs = np.sqrt(np.repeat(psd, 2))
    res = [np.zeros(len(t)) for t in toas_list]
    fourier = np.zeros((P, 2, components))
    for i in range(components):
        orf_corr_sin = L @ z[i, 0]
        orf_corr_cos = L @ z[i, 1]
        for n in range(P):
            fourier[n, 0, i] = orf_corr_cos[n] * coeffs[2 * i] / df[i] ** 0.5
            fourier[n, 1, i] = orf_corr_sin[n] * coeffs[2 * i + 1] / df[i] ** 0.5
            ch = (freqf / freqs_list[n]) ** idx
            res[n] += orf_corr_cos[n] * ch * df[i] ** 0.5 * coeffs[2 * i] * np.cos(2 * np.pi * f[i] * toas_list[n])
            res[n] += orf_corr_sin[n] * ch * df[i] ** 0.5 * coeffs[2 * i + 1] * np.sin(2 * np.pi * f[i] * toas_list[n])
    return res, fourier


def redraw_loop(toas_list, freqs_list, segs, residuals, stored, rs, freqf=1400.0):
    """One re-drawn realization of an array's noise model with the reference's own operations, in its order and at
    its cost (the CPU baseline of SURVEY.md §8(d)(i)):
      * per pulsar, per per-pulsar GP (fake_pta.py:266-267, 370-387): residuals -= reconstruct_signal of the stored
        coefficients (:538-545); coeffs = normal(0, sqrt(repeat(psd, 2))); two elementwise passes per mode, each
        recomputing (freqf / nu)**idx;
      * per common GP (correlated_noises.py:133-134, 146-160): residuals -= reconstruct_signal on every pulsar; per
        mode two multivariate_normal draws (each factors the ORF by SVD, numpy's method) and two elementwise passes
        per pulsar.
    segs: dicts kind (0 per pulsar: f, psd [P, N]; 1 common: f, psd [N], orf [P, P]), idx. residuals: list of
    per-pulsar arrays (updated in place). stored: {(segment, pulsar): fourier [2, N]} of the previous realization
    (updated in place; empty on the first call). rs: numpy.random.RandomState (the reference's legacy stream)."""
    P = len(toas_list)
    for p in range(P):
        toas, freqs, res = toas_list[p], freqs_list[p], residuals[p]
        for si, sg in enumerate(segs):
            if sg["kind"] != 0:
                continue
            f, psd, idx = sg["f"][p], sg["psd"][p], sg["idx"]
            if (si, p) in stored:
                res -= reconstruct_loop(toas, freqs, f, stored[(si, p)], idx, freqf)
            df = delta_f(f)
            psd2 = np.repeat(psd, 2)
            coeffs = rs.normal(loc=0., scale=np.sqrt(psd2))
            stored[(si, p)] = np.vstack((coeffs[::2] / df ** 0.5, coeffs[1::2] / df ** 0.5))
            mask = np.ones(len(toas), dtype=bool)  # backend=None: an all-true mask, indexed as at :386-387
            for i in range(len(f)):
                res[mask] += (freqf / freqs) ** idx * df[i] ** 0.5 * coeffs[2 * i] * np.cos(2 * np.pi * f[i] * toas[mask])
                res[mask] += (freqf / freqs) ** idx * df[i] ** 0.5 * coeffs[2 * i + 1] * np.sin(2 * np.pi * f[i] * toas[mask])
    for si, sg in enumerate(segs):
        if sg["kind"] != 1:
            continue
        f, psd, idx, orf = sg["f"], sg["psd"], sg["idx"], sg["orf"]
        for p in range(P):
            if (si, p) in stored:
                residuals[p] -= reconstruct_loop(toas_list[p], freqs_list[p], f, stored[(si, p)], idx, freqf)
            stored[(si, p)] = np.zeros((2, len(f)))
        df = delta_f(f)
        coeffs = np.sqrt(np.repeat(psd, 2))
        for i in range(len(f)):
            x_sin = rs.multivariate_normal(mean=np.zeros(P), cov=orf)
            x_cos = rs.multivariate_normal(mean=np.zeros(P), cov=orf)
            for n in range(P):
                stored[(si, n)][0, i] = x_cos[n] * coeffs[2 * i] / df[i] ** 0.5
                stored[(si, n)][1, i] = x_sin[n] * coeffs[2 * i + 1] / df[i] ** 0.5
                t, nu = toas_list[n], freqs_list[n]
                residuals[n] += x_cos[n] * (freqf / nu) ** idx * df[i] ** 0.5 * coeffs[2 * i] * np.cos(2 * np.pi * f[i] * t)
                residuals[n] += x_sin[n] * (freqf / nu) ** idx * df[i] ** 0.5 * coeffs[2 * i + 1] * np.sin(2 * np.pi * f[i] * t)
    return residuals


# ----------------------------------------------------------------------------- white noise / ECORR

def white_sigma(toaerrs, backend_flags, efac, log10_tnequad):
    """fakepta/fake_pta.py:214-217: sigma^2 = efac_b^2 sigma_toa^2 + 10^(2 log10_tnequad_b).
    efac / log10_tnequad: dicts backend -> value."""
    s2 = np.zeros(len(toaerrs))
    for b in np.unique(backend_flags):
        m = backend_flags == b
        s2[m] = efac[b] ** 2 * toaerrs[m] ** 2 + 10 ** (2 * log10_tnequad[b])
    return s2 ** 0.5


def quantise_ecorr(toas, backend_flags, backends, dt=1):
    """fakepta/fake_pta.py:232-253 verbatim semantics, including defect D2 (the final block
    of every backend is never appended)."""
    times = toas - toas[0]
    out = []
    dt *= 24 * 3600
    for backend in backends:
        b_idx = np.arange(len(times))[backend_flags == backend]
        t0 = times[b_idx[0]]
        q_i = [b_idx[0]]
        for n in b_idx[1:]:
            if times[n] - t0 < dt:
                q_i.append(n)
            else:
                t0 = times[n]
                out.append(np.array(q_i))
                q_i = [n]
    return out


def ecorr_blocks(toas, backend_flags, backends, dt=1):
    """The build's ECORR epochs: quantise_ecorr's greedy 1-day blocks per backend, WITH the
    final block appended (fixes D2)."""
    times = toas - toas[0]
    out = []
    dt *= 24 * 3600
    for backend in backends:
        b_idx = np.arange(len(times))[backend_flags == backend]
        if len(b_idx) == 0:
            continue
        t0 = times[b_idx[0]]
        q_i = [b_idx[0]]
        for n in b_idx[1:]:
            if times[n] - t0 < dt:
                q_i.append(n)
            else:
                t0 = times[n]
                out.append(np.array(q_i))
                q_i = [n]
        out.append(np.array(q_i))
    return out


# ----------------------------------------------------------------------------- Philox4x32-10

PHILOX_M0, PHILOX_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
PHILOX_W0, PHILOX_W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr, key):
    """Random123 Philox4x32-10. ctr: uint32 [..., 4]; key: uint32 [..., 2] (broadcast)."""
    c = [np.asarray(ctr[..., i], dtype=np.uint64) for i in range(4)]
    k0 = np.asarray(key[..., 0], dtype=np.uint64)
    k1 = np.asarray(key[..., 1], dtype=np.uint64)
    for _ in range(10):
        p0 = PHILOX_M0 * c[0]
        p1 = PHILOX_M1 * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & MASK32, p1 & MASK32,
             ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & MASK32, p0 & MASK32]
        k0 = (k0 + np.uint64(PHILOX_W0)) & MASK32
        k1 = (k1 + np.uint64(PHILOX_W1)) & MASK32
    return np.stack([x.astype(np.uint32) for x in c], axis=-1)


def box_muller(x):
    """uint32 [..., 4] -> two standard normals [..., 2] with 53-bit uniforms (the round-1/2 mapping; kept for
    reference and statistical comparison, no longer used by any stream):
    u1 = ((x0|x1<<32) >> 11) + 1) * 2^-53 in (0, 1], u2 = ((x2|x3<<32) >> 11) * 2^-53 in [0, 1),
    z0 = sqrt(-2 ln u1) cos(2 pi u2), z1 = sqrt(-2 ln u1) sin(2 pi u2)."""
    x = x.astype(np.uint64)
    a = x[..., 0] | (x[..., 1] << np.uint64(32))
    b = x[..., 2] | (x[..., 3] << np.uint64(32))
    u1 = ((a >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
    u2 = (b >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
    r = np.sqrt(-2.0 * np.log(u1))
    th = TWO_PI * u2
    return np.stack([r * np.cos(th), r * np.sin(th)], axis=-1)


# The build's uniform -> normal map (philox.h normals4): two Box-Muller pairs per Philox call from 32-bit uniforms
# u1 = (a + 1) 2^-32 in (0, 1], u2 = b 2^-32 in [0, 1) (as cuRAND's normal2), with the logarithm and the sine / cosine
# evaluated by fixed fp64 polynomials that the device restates operation for operation (agreement to a few ulp; the
# polynomials are accurate to ~3e-14 relative; the device's quotient in the logarithm and its square root come from
# v_rcp_f64 / v_rsq_f64 plus Newton steps, within an ulp of the IEEE results taken here). |z| <= sqrt(64 ln 2) = 6.66.
SQRT_HALF = 0.7071067811865476
LN2_HI, LN2_LO = 6.93147180369123816490e-01, 1.90821492927058770002e-10
_LOG_C = (1.0 / 3.0, 1.0 / 5.0, 1.0 / 7.0, 1.0 / 9.0, 1.0 / 11.0, 1.0 / 13.0, 1.0 / 15.0)
_SIN_C = (-1.0 / 6.0, 1.0 / 120.0, -1.0 / 5040.0, 1.0 / 362880.0, -1.0 / 39916800.0, 1.0 / 6227020800.0)
_COS_C = (-1.0 / 2.0, 1.0 / 24.0, -1.0 / 720.0, 1.0 / 40320.0, -1.0 / 3628800.0, 1.0 / 479001600.0,
          -1.0 / 87178291200.0)


def _horner(x, coefs):
    acc = np.full_like(x, coefs[-1])
    for c in coefs[-2::-1]:
        acc = c + x * acc
    return acc


def bm_log_u32(a):
    """log((a + 1) 2^-32) for uint32 a: frexp to m in [sqrt(1/2), sqrt(2)), log m = 2 atanh((m - 1) / (m + 1)) by its
    series to s^15, plus (e - 32) ln 2 in two parts."""
    n = np.asarray(a, dtype=np.uint32).astype(np.float64) + 1.0
    m, e = np.frexp(n)
    low = m < SQRT_HALF
    m = np.where(low, 2.0 * m, m)
    e = np.where(low, e - 1, e)
    k = (e - 32).astype(np.float64)
    sv = (m - 1.0) / (m + 1.0)
    s2 = sv * sv
    p = s2 * _horner(s2, _LOG_C)
    lm = 2.0 * sv + 2.0 * sv * p
    return k * LN2_HI + (k * LN2_LO + lm)


def bm_sincos2pi_u32(b):
    """(sin, cos)(2 pi b 2^-32): nearest quarter turn q, remainder a = 2 pi (u - q / 4) in [-pi/4, pi/4] by Taylor
    polynomials (sin to a^13, cos to a^14), then the quadrant."""
    u = np.asarray(b, dtype=np.uint32).astype(np.float64) * 2.0 ** -32
    q = np.rint(4.0 * u)
    y = u - 0.25 * q
    a = y * TWO_PI
    x2 = a * a
    sa = a + a * x2 * _horner(x2, _SIN_C)
    ca = 1.0 + x2 * _horner(x2, _COS_C)
    qi = q.astype(np.int64) & 3
    sn = np.select([qi == 0, qi == 1, qi == 2], [sa, ca, -sa], -ca)
    cs = np.select([qi == 0, qi == 1, qi == 2], [ca, -sa, -ca], sa)
    return sn, cs


def normals4(x):
    """uint32 [..., 4] (one Philox4x32-10 output) -> four standard normals [..., 4]: (z0, z1) from (x0, x1),
    (z2, z3) from (x2, x3); z0 = r cos, z1 = r sin, r = sqrt(-2 log u1)."""
    x = np.asarray(x, dtype=np.uint32)
    out = []
    for i in (0, 2):
        r = np.sqrt(-2.0 * bm_log_u32(x[..., i]))
        sn, cs = bm_sincos2pi_u32(x[..., i + 1])
        out += [r * cs, r * sn]
    return np.stack(out, axis=-1)


# stream identifiers (counter word 1 / 2) for the non-GP draws
WHITE_PSR_WORD = 0xFFFFFFFF
WHITE_STREAM = 0xFFFFFFF0
ECORR_STREAM = 0xFFFFFFF1
DENSE_STREAM = 0xFFFFFFF2


def seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return np.array([seed & 0xFFFFFFFF, seed >> 32], dtype=np.uint32)


def gp_normals(seed, reals, p, seg, n_modes):
    """(z_cos, z_sin) for modes 0..N-1 of pulsar p, segment seg, global realizations `reals`: one Philox call per
    (mode, pulsar, segment, realization pair), ctr = (mode, pulsar, segment, g >> 1); realization g takes normals
    (2 (g & 1), 2 (g & 1) + 1) of it. Returns [R, N, 2]."""
    reals = np.asarray(reals, dtype=np.uint64)
    k = np.arange(n_modes, dtype=np.uint32)
    ctr = np.zeros((len(reals), n_modes, 4), dtype=np.uint32)
    ctr[..., 0] = k[None, :]
    ctr[..., 1] = p
    ctr[..., 2] = seg
    ctr[..., 3] = (reals >> np.uint64(1)).astype(np.uint32)[:, None]
    z = normals4(philox4x32_10(ctr, seed_key(seed)))  # [R, N, 4]
    h = 2 * (reals & np.uint64(1)).astype(np.int64)[:, None, None]
    return np.concatenate([np.take_along_axis(z, np.broadcast_to(h, z.shape[:-1] + (1,)), axis=-1),
                           np.take_along_axis(z, np.broadcast_to(h + 1, z.shape[:-1] + (1,)), axis=-1)], axis=-1)


def quad_normals(seed, reals, n, stream):
    """One normal per (realization g, index i) from a stream paired over both: ctr = (i >> 1, 0xFFFFFFFF, stream,
    g >> 1), normal 2 (i & 1) + (g & 1) of the call. White noise (index = TOA, WHITE_STREAM), ECORR epochs (index =
    epoch, ECORR_STREAM) and the dense draws (index = TOA, DENSE_STREAM). Returns [len(reals), n]."""
    reals = np.asarray(reals, dtype=np.uint64)
    t = np.arange(n, dtype=np.uint64)
    ctr = np.zeros((len(reals), n, 4), dtype=np.uint32)
    ctr[..., 0] = (t >> np.uint64(1)).astype(np.uint32)[None, :]
    ctr[..., 1] = WHITE_PSR_WORD
    ctr[..., 2] = stream
    ctr[..., 3] = (reals >> np.uint64(1)).astype(np.uint32)[:, None]
    z = normals4(philox4x32_10(ctr, seed_key(seed)))
    pick = 2 * (t & np.uint64(1)).astype(np.int64)[None, :] + (reals & np.uint64(1)).astype(np.int64)[:, None]
    return np.take_along_axis(z, pick[..., None], axis=-1)[..., 0]


def white_normals_rpairs(seed, reals, n_toa, stream=WHITE_STREAM):
    """White-noise normals [len(reals), n_toa] (quad_normals on the white stream)."""
    return quad_normals(seed, reals, n_toa, stream)


def white_normals(seed, reals, n, stream=WHITE_STREAM):
    """Normals of an indexed stream, e.g. the ECORR epochs (quad_normals)."""
    return quad_normals(seed, reals, n, stream)


# ----------------------------------------------------------------------------- batch semantics

class Segment:
    """One GP signal of the batch layout.
    kind 0 (per pulsar): w [P, N], amp [P, N];  kind 1 (common): w [N], amp [N], L [P, P].
    w = 2*pi*f (rad/s); amp = sqrt(S * df) (the standard deviation of each coefficient)."""

    def __init__(self, kind, w, amp, idx=0.0, freqf=1400.0, L=None, mask=None):
        self.kind, self.w, self.amp = kind, np.asarray(w, float), np.asarray(amp, float)
        self.idx, self.freqf, self.L, self.mask = float(idx), float(freqf), L, mask

    @property
    def n_modes(self):
        return self.w.shape[-1]


def batch_coefficients(segments, n_psr, seed, real0, n_real, z_override=None):
    """Coefficients a[s][R, P, N, 2] (cos, sin) of every segment for realizations
    real0..real0+n_real-1. z_override: optional dict s -> z [R, P, N, 2] (validation mode)."""
    reals = np.arange(real0, real0 + n_real)
    out = []
    for s, seg in enumerate(segments):
        if z_override is not None and s in z_override:
            z = z_override[s]
        else:
            z = np.stack([gp_normals(seed, reals, p, s, seg.n_modes) for p in range(n_psr)], axis=1)
        if seg.kind == 0:
            a = seg.amp[None, :, :, None] * z
        else:
            x = np.einsum("pq,rqnc->rpnc", seg.L, z)
            a = seg.amp[None, None, :, None] * x
        out.append(a)
    return out


def batch_synth(offs, toas, freqs, segments, seed, real0, n_real, sigma=None, block_of=None,
                ecorr_sigma=None, z_override=None):
    """Full batch semantics: out [n_real, n_toa_total]."""
    P = len(offs) - 1
    coeffs = batch_coefficients(segments, P, seed, real0, n_real, z_override)
    out = np.zeros((n_real, offs[-1]))
    for s, seg in enumerate(segments):
        a = coeffs[s]
        for p in range(P):
            sl = slice(offs[p], offs[p + 1])
            w = seg.w[p] if seg.kind == 0 else seg.w
            ph = np.outer(toas[sl], w)
            ch = (seg.freqf / freqs[sl]) ** seg.idx
            if seg.mask is not None:
                ch = ch * seg.mask[sl]
            out[:, sl] += ch[None, :] * (a[:, p, :, 0] @ np.cos(ph).T + a[:, p, :, 1] @ np.sin(ph).T)
    reals = np.arange(real0, real0 + n_real)
    if sigma is not None:
        out += sigma[None, :] * white_normals_rpairs(seed, reals, offs[-1])
    if block_of is not None and ecorr_sigma is not None and len(ecorr_sigma):
        zb = white_normals(seed, reals, len(ecorr_sigma), ECORR_STREAM)
        has = block_of >= 0
        out[:, has] += ecorr_sigma[block_of[has]][None, :] * zb[:, block_of[has]]
    return out


# ----------------------------------------------------------------------------- dense covariance
def dense_cov_signal(toas, freqs, f, psd, idx, freqf=1400.0):
    """make_time_correlated_noise_cov (fake_pta.py:389-420): basis [n, 2N] with the chromatic
    factor, cov = basis diag(repeat(psd df, 2)) basis^T."""
    df = np.diff(np.append(0, f))
    w = np.repeat(psd * df, 2)
    basis = np.zeros((len(toas), 2 * len(f)))
    ch = (freqf / freqs) ** idx
    for i in range(len(f)):
        basis[:, 2 * i] = ch * np.cos(2 * np.pi * f[i] * toas)
        basis[:, 2 * i + 1] = ch * np.sin(2 * np.pi * f[i] * toas)
    return np.dot(basis, np.dot(np.diag(w), basis.T))


def dense_cov(toas, freqs, signals, freqf=1400.0):
    """red part of make_noise_covariance_matrix (fake_pta.py:505-512): sum over (f, psd, idx)."""
    red = np.zeros((len(toas), len(toas)))
    for f, psd, idx in signals:
        red += dense_cov_signal(toas, freqs, f, psd, idx, freqf)
    return red


def wiener_reference(white_cov, red_cov, residuals):
    """draw_noise_model(residuals) (fake_pta.py:516-523), the reference's explicit-inverse form."""
    cov = np.diag(white_cov) + red_cov
    return np.dot(red_cov.T, np.dot(np.linalg.inv(cov), residuals))


def dense_draws(cov, seed, real0, n_real):
    """Batched N(0, cov) draws of this build: x_r = L z_r with L = cholesky(cov) and z the
    DENSE_STREAM normals (ctr = (toa, 0xFFFFFFFF, 0xFFFFFFF2, g >> 1), pick [g & 1])."""
    L = np.linalg.cholesky(cov)
    z = white_normals_rpairs(seed, np.arange(real0, real0 + n_real), cov.shape[0], stream=DENSE_STREAM)
    return z @ L.T


# ----------------------------------------------------------------------------- gridded synthesis model
# Numpy model of the library's gridded path (grid.hip, FPTA_OPT_SYNTH_PATH 4): the same sum as
# gp_synth_vec on a harmonic grid f_k = k f_1 (fake_pta.py:264, correlated_noises.py:120),
# factored as a type-2 non-uniform FFT. Not a reference function: it documents the approximation
# and lets the CPU suite check its error bound (tests/test_oracle_golden.py).
def es_kernel(z, beta):
    """Exponential of semicircle phi(z) = exp(beta (sqrt(1 - z^2) - 1)) on |z| < 1, else 0."""
    z = np.asarray(z, dtype=float)
    s = 1.0 - z * z
    return np.where(s > 0, np.exp(beta * (np.sqrt(np.maximum(s, 0.0)) - 1.0)), 0.0)


def grid_params(n_modes, w=13, sigma=2.0):
    """Grid size nf >= sigma (2N + 1) (even, >= 2w + 2) and kernel shape beta for width w."""
    nf = int(np.ceil(sigma * (2 * n_modes + 1)))
    nf += nf & 1
    nf = max(nf, 2 * w + 2)
    beta = 0.98 * np.pi * w * (1.0 - 0.5 / sigma)
    return nf, beta


def grid_deconvolution(n_modes, nf, w, beta, n_quad=256):
    """q_k = (2 pi / nf) / phi_hat(k), phi_hat(k) = alpha int_{-1}^{1} phi(z) cos(k alpha z) dz with
    alpha = pi w / nf (Gauss-Legendre quadrature), k = 1..N."""
    alpha = np.pi * w / nf
    x, wt = np.polynomial.legendre.leggauss(n_quad)
    k = np.arange(1, n_modes + 1)
    ph = alpha * (np.cos(np.outer(k, alpha * x)) @ (wt * es_kernel(x, beta)))
    return (2.0 * np.pi / nf) / ph


def grid_synth(toas, freqs, w0, amp_cos, amp_sin, idx, freqf=1400.0, w=13, sigma=2.0):
    """sum_k chrom(t) (amp_cos_k cos(k w0 t) + amp_sin_k sin(k w0 t)) through the grid:
    g_j = sum_k q_k (amp_cos_k cos(2 pi k j / nf) + amp_sin_k sin(2 pi k j / nf)), then
    r(t) = chrom(t) sum_{i<w} phi((u - J - i) / (w/2)) g_{(J + i) mod nf}, u = w0 t / h, h = 2 pi / nf,
    J = floor(u - w/2) + 1. amp_* of shape [N] or [R, N]."""
    amp_cos = np.atleast_2d(amp_cos)
    amp_sin = np.atleast_2d(amp_sin)
    N = amp_cos.shape[-1]
    nf, beta = grid_params(N, w, sigma)
    q = grid_deconvolution(N, nf, w, beta)
    k = np.arange(1, N + 1)
    ang = TWO_PI * ((np.outer(np.arange(nf), k)) % nf) / nf
    g = (amp_cos * q) @ np.cos(ang).T + (amp_sin * q) @ np.sin(ang).T  # [R, nf]
    u = (w0 * np.asarray(toas)) / (TWO_PI / nf)
    J = np.floor(u - 0.5 * w).astype(np.int64) + 1
    out = np.zeros((amp_cos.shape[0], len(toas)))
    for i in range(w):
        out += es_kernel((u - (J + i)) / (0.5 * w), beta)[None, :] * g[:, (J + i) % nf]
    return chromatic(freqs, idx, freqf)[None, :] * out
