"""Power-spectral-density models, S(f) in s^3 (drop-in for fakepta/spectrum.py:12-86).

The forms are ENTERPRISE's gp_priors: a characteristic strain h_c(f) converted to a
residual PSD as h_c^2 / (12 pi^2 f^3). They are evaluated on the host (O(n_modes)); the
kernels receive sqrt(S * df) per mode.
"""
import numpy as np

from .constants import fyr

__all__ = ["powerlaw", "turnover", "t_process", "t_process_adapt", "turnover_knee", "broken_powerlaw"]


def powerlaw(f, log10_A, gamma):
    """fakepta/spectrum.py:12-15"""
    amp2 = (10 ** log10_A) ** 2
    return amp2 / (12.0 * np.pi ** 2) * fyr ** (gamma - 3) * f ** (-gamma)


def _hc2_to_psd(hc, f):
    return hc ** 2 / 12 / np.pi ** 2 / f ** 3


def turnover(f, log10_A=-15, gamma=4.33, lf0=-8.5, kappa=10 / 3, beta=0.5):
    """fakepta/spectrum.py:18-20 — low-frequency turnover at f0 = 10^lf0."""
    slope = (f / fyr) ** ((3 - gamma) / 2)
    bend = (1 + (10 ** lf0 / f) ** kappa) ** beta
    return _hc2_to_psd(10 ** log10_A * slope / bend, f)


def t_process(f, log10_A=-15, gamma=4.33, alphas=None):
    """fakepta/spectrum.py:23-29 — power law times per-frequency weights."""
    weights = np.ones_like(f) if alphas is None else alphas
    return powerlaw(f, log10_A=log10_A, gamma=gamma) * weights


def t_process_adapt(f, log10_A=-15, gamma=4.33, alphas_adapt=None, nfreq=None):
    """fakepta/spectrum.py:32-46 — weight on one (rounded) frequency bin, or per-bin weights."""
    if alphas_adapt is None:
        weights = np.ones_like(f)
    elif nfreq is None:
        weights = alphas_adapt
    else:
        weights = np.ones_like(f)
        weights[int(np.rint(nfreq))] = alphas_adapt
    return powerlaw(f, log10_A=log10_A, gamma=gamma) * weights


def turnover_knee(f, log10_A, gamma, lfb, lfk, kappa, delta):
    """fakepta/spectrum.py:49-66 — turnover at 10^lfb plus a high-frequency knee at 10^lfk."""
    slope = (f / fyr) ** ((3 - gamma) / 2)
    knee = (1.0 + (f / 10 ** lfk)) ** delta
    bend = np.sqrt(1 + (10 ** lfb / f) ** kappa)
    return _hc2_to_psd(10 ** log10_A * slope * knee / bend, f)


def broken_powerlaw(f, log10_A, gamma, delta, log10_fb, kappa=0.1):
    """fakepta/spectrum.py:69-86 — slope delta below 10^log10_fb, gamma above."""
    slope = (f / fyr) ** ((3 - gamma) / 2)
    brk = (1 + (f / 10 ** log10_fb) ** (1 / kappa)) ** (kappa * (gamma - delta) / 2)
    return _hc2_to_psd(10 ** log10_A * slope * brk, f)
