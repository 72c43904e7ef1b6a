"""Drop-in for fakepta/correlated_noises.py: inter-pulsar-correlated common GPs.

add_common_correlated_noise keeps the reference's host side (PSD, noisedict, signal_model,
np.random draws in multivariate_normal's order: per mode the sin vector, then the cos
vector), computes the same SVD square root of the ORF that numpy's multivariate_normal
uses, and hands the draws to the GPU, which applies the ORF factor and evaluates every
pulsar's Fourier sum (libfakepta_amd: fpta_common_accumulate).
"""
import importlib
import inspect

import numpy as np

from fakepta_amd import _capi
from . import spectrum as _spectrum_module
from .fake_pta import Pulsar  # noqa: F401  (reference module namespace)
from .fake_pta import reconstruct_array

spec = {name: fn for name, fn in inspect.getmembers(_spectrum_module, inspect.isfunction)
        if name in _spectrum_module.__all__}


# ----------------------------------------------------------------------------- estimators
def get_correlation(psr_a, psr_b, res_a, res_b):
    """Zero-lag cross-correlation and angular separation (correlated_noises.py:14-19)."""
    return np.dot(res_a, res_b) / len(res_a), np.arccos(np.dot(psr_a.pos, psr_b.pos))


def get_correlations(psrs, res):
    """All pairs i >= j: cross-correlations, angles, auto-correlations (correlated_noises.py:21-34)."""
    corrs, angles, autos = [], [], []
    for i in range(len(psrs)):
        for j in range(i + 1):
            c, a = get_correlation(psrs[i], psrs[j], res[i], res[j])
            if i == j:
                autos.append(c)
            else:
                corrs.append(c)
                angles.append(a)
    return np.array(corrs), np.array(angles), np.array(autos)


def bin_curve(corrs, angles, bins):
    """Mean/std of correlations in equal angular bins over (0, pi) (correlated_noises.py:36-47)."""
    edges = np.linspace(0., np.pi, bins + 1)
    centres = edges[:-1] + 0.5 * (edges[1] - edges[0])
    mean, std = [], []
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = (angles > lo) & (angles < hi)
        mean.append(np.mean(corrs[sel]))
        std.append(np.std(corrs[sel]))
    return np.array(mean), np.array(std), centres


# ----------------------------------------------------------------------------- ORFs
def _positions(psrs):
    return np.array([p.pos for p in psrs])


def create_gw_antenna_pattern(pos, gwtheta, gwphi):
    """F+, Fx and cos(mu) of a pulsar for GW sources at (gwtheta, gwphi) (correlated_noises.py:50-60)."""
    m = np.array([np.sin(gwphi), -np.cos(gwphi), np.zeros(len(gwphi))]).T
    n = np.array([-np.cos(gwtheta) * np.cos(gwphi), -np.cos(gwtheta) * np.sin(gwphi), np.sin(gwtheta)]).T
    omhat = np.array([-np.sin(gwtheta) * np.cos(gwphi), -np.sin(gwtheta) * np.sin(gwphi), -np.cos(gwtheta)]).T
    mp, nq, op = m @ pos, n @ pos, omhat @ pos
    return 0.5 * (mp ** 2 - nq ** 2) / (1 + op), (mp * nq) / (1 + op), -op


def hd(psrs):
    """Hellings-Downs: 1.5 x ln x - x/4 + 1/2, x = (1 - cos zeta)/2, unit diagonal
    (correlated_noises.py:62-71). Coincident pulsars give NaN, as in the reference (D8)."""
    pos = _positions(psrs)
    with np.errstate(divide='ignore', invalid='ignore'):
        x = (1 - pos @ pos.T) / 2
        orf = 1.5 * x * np.log(x) - 0.25 * x + 0.5
    np.fill_diagonal(orf, 1.)
    return orf


def anisotropic(psrs, h_map):
    """ORF of an anisotropic GWB given as a healpy map (correlated_noises.py:73-89). Needs healpy."""
    hp = importlib.import_module('healpy')
    npix = len(h_map)
    gwtheta, gwphi = hp.pix2ang(hp.npix2nside(npix), np.arange(npix), nest=False)
    fp, fc = [], []
    for psr in psrs:
        a, b, _ = create_gw_antenna_pattern(psr.pos, gwtheta, gwphi)
        fp.append(a)
        fc.append(b)
    fp, fc = np.array(fp), np.array(fc)
    orf = 1.5 * ((fp * h_map) @ fp.T + (fc * h_map) @ fc.T) / npix
    orf[np.diag_indices_from(orf)] *= 2.0
    return orf


def monopole(psrs):
    """(correlated_noises.py:91-93)"""
    return np.ones((len(psrs), len(psrs)))


def dipole(psrs):
    """cos zeta, unit diagonal (correlated_noises.py:95-104)."""
    pos = _positions(psrs)
    orf = pos @ pos.T
    np.fill_diagonal(orf, 1.)
    return orf


def curn(psrs):
    """Uncorrelated common process (correlated_noises.py:106-108)."""
    return np.eye(len(psrs))


ORF_FUNCS = {'hd': hd, 'monopole': monopole, 'dipole': dipole, 'curn': curn}


def orf_matrix(psrs, orf, h_map=None):
    if isinstance(orf, np.ndarray):
        return orf
    if orf in ORF_FUNCS:
        return ORF_FUNCS[orf](psrs)
    if orf == 'anisotropic':
        return anisotropic(psrs, h_map)
    raise ValueError(f'unknown ORF {orf!r}')


def orf_factor(orf_mat):
    """Square root L (L L^T = ORF) exactly as numpy's legacy multivariate_normal builds it:
    x = z @ (sqrt(s)[:, None] * vt) from svd(cov). Works for the singular monopole / dipole
    ORFs, where a Cholesky factor does not exist. Returned as L = M^T so x = L z."""
    _, s, vt = np.linalg.svd(orf_mat)
    return np.ascontiguousarray((np.sqrt(s)[:, None] * vt).T)


# ----------------------------------------------------------------------------- injection
def add_common_correlated_noise(psrs, orf='hd', spectrum='powerlaw', name='gw', idx=0, components=30, freqf=1400,
                                custom_psd=None, f_psd=None, h_map=None, **kwargs):
    """Common GP with inter-pulsar correlation `orf` on the array's global frequency grid
    (correlated_noises.py:111-160)."""
    signal_name = name + '_common' if name is not None else 'common'
    tspan = np.amax([p.toas.max() for p in psrs]) - np.amin([p.toas.min() for p in psrs])
    if f_psd is None:
        f_psd = np.arange(1, components + 1) / tspan
    f_psd = np.asarray(f_psd, dtype=float)
    df = np.diff(np.append(0., f_psd))
    if spectrum == 'custom':
        assert len(custom_psd) == len(f_psd), ('"custom_psd" and "f_psd" must be same length. The frequencies '
                                               '"f_psd" correspond to frequencies where the "custom_psd" is '
                                               'evaluated.')
        psd = np.asarray(custom_psd, dtype=float)
    elif spectrum in spec:
        psd = spec[spectrum](f_psd, **kwargs)
        for p in psrs:
            p.update_noisedict(signal_name, kwargs)
    else:
        raise ValueError(f'unknown spectrum {spectrum!r}')
    # the reference sizes `fourier` / `nbin` by `components` and loops range(components) over the first modes of
    # f_psd, storing the full f and psd (correlated_noises.py:140-160); with fewer frequencies than components it
    # injects every mode, draws one more (sin, cos) pair and fails on coeffs[2 * len(f_psd)] (:157)
    n_modes = min(int(components), len(f_psd))
    # replace-on-reinject (correlated_noises.py:133-134), all pulsars in one GPU launch
    if any(signal_name in p.signal_model for p in psrs):
        old = reconstruct_array(psrs, [signal_name])
        for p, r in zip(psrs, old):
            p.residuals -= r
    for p in psrs:
        p.signal_model[signal_name] = {'orf': orf, 'spectrum': spectrum, 'hmap': h_map, 'f': f_psd, 'psd': psd,
                                       'fourier': np.zeros((2, components)), 'nbin': components, 'idx': idx}
    amp0 = np.sqrt(np.repeat(psd, 2))[0::2][:n_modes]  # coeffs[2i] of correlated_noises.py:147
    sq_df = df[:n_modes] ** 0.5
    L = orf_factor(orf_matrix(psrs, orf, h_map))
    P = len(psrs)
    # multivariate_normal(mean=0, cov=orf) draws standard_normal(P) per call: sin first, then cos
    z = np.empty((n_modes, 2, P))
    for i in range(n_modes):
        z[i, 0] = np.random.standard_normal(P)
        z[i, 1] = np.random.standard_normal(P)
    offs = np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])]).astype(np.int64)
    res = np.concatenate([p.residuals for p in psrs])
    if n_modes:
        x = _capi.get_context().common_accumulate(offs, np.concatenate([p.toas for p in psrs]),
                                                  np.concatenate([p.freqs for p in psrs]), f_psd[:n_modes],
                                                  sq_df * amp0, float(idx), float(freqf), L, z, res)
    for n, p in enumerate(psrs):
        p.residuals[:] = res[offs[n]:offs[n + 1]]
        if n_modes:
            p.signal_model[signal_name]['fourier'][0, :n_modes] = x[:, 0, n] * amp0 / sq_df
            p.signal_model[signal_name]['fourier'][1, :n_modes] = x[:, 1, n] * amp0 / sq_df
    if components > n_modes:
        np.random.standard_normal(P)
        np.random.standard_normal(P)
        raise IndexError(f'index {2 * len(f_psd)} is out of bounds for axis 0 with size {2 * len(f_psd)}')

def add_roemer_delay(psrs, planet, d_mass=0., d_Om=0., d_omega=0., d_inc=0., d_a=0., d_e=0., d_l0=0.):
    """Ephemeris-error Roemer delay (correlated_noises.py:163-172). Deterministic, not part of the
    accelerated path: needs a Pulsar built with an `ephem` object exposing roemer_delay()."""
    for p in psrs:
        if not hasattr(p, 'ephem'):
            print('"ephem" not found in pulsar', p.name)
            return
    for p in psrs:
        p.residuals += p.ephem.roemer_delay(p.toas, p.pos, planet, d_mass, d_Om, d_omega, d_inc, d_a, d_e, d_l0)
