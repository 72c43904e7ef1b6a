"""Batched realizations: many independent draws of an array's noise model on one MI355X.

The reference produces one realization per Python call (make_fake_array / add_* /
add_common_correlated_noise, a loop over pulsars and modes). BatchSimulator takes the noise
model an array already carries (each Pulsar's signal_model and noisedict, as left by
make_fake_array or the add_* injectors) and re-draws it R times on the device:

    Philox4x32-10 draws -> ORF mixing -> fused basis/contraction -> white/ECORR

Realization r of seed s is the same whatever the batch split or number of GPUs (the Philox
counter carries the global realization index), so realizations shard across ranks with no
data-path collective. The draws are not numpy's MT19937 stream (SURVEY.md §7 'RNG parity');
the oracle (oracle/fakepta_oracle.py: batch_synth) restates the exact semantics.
"""
import numpy as np

from . import _capi
from .correlated_noises import bin_curve, orf_factor, orf_matrix

GP_NAMES = ("red_noise", "dm_gp", "chrom_gp")


def _df(f):
    return np.diff(np.append(0.0, f))


def batch_factor(orf_mat):
    """Square root of the ORF for batched draws: the lower Cholesky factor when the ORF is
    positive definite (HD, curn: triangular mixing on device, half the FLOPs), otherwise the SVD
    factor numpy's multivariate_normal uses (singular monopole / dipole ORFs). Any L with
    L L^T = ORF gives the reference's distribution; the drop-in path keeps numpy's exact factor."""
    try:
        return np.ascontiguousarray(np.linalg.cholesky(orf_mat))
    except np.linalg.LinAlgError:
        return orf_factor(orf_mat)


class BatchSimulator:
    """Device-resident noise model of an array of Pulsar objects.

    signals: names to include (default: every GP signal found in the pulsars' signal_model:
             red_noise, dm_gp, chrom_gp, '*system_noise*' and '*common*').
    white:   include EFAC/EQUAD white noise from each pulsar's noisedict.
    ecorr:   include ECORR epochs (ENTERPRISE convention 10^(2 log10_ecorr)).
    """

    def __init__(self, psrs, signals=None, white=True, ecorr=False, device=None, ctx=None):
        self.psrs = psrs
        self.ctx = ctx if ctx is not None else _capi.get_context(device)
        self.offs = np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])]).astype(np.int64)
        self.toas = np.concatenate([p.toas for p in psrs])
        self.freqs = np.concatenate([p.freqs for p in psrs])
        self.ctx.batch_set_toas(self.offs, self.toas, self.freqs)
        self.segments = []  # (name, kind, f, amp, idx, L, mask) — host copy for checking/reporting
        names = signals
        if names is None:
            names = []
            for p in psrs:
                for s in p.signal_model:
                    if s not in names and (s in GP_NAMES or "common" in s or "system_noise" in s):
                        names.append(s)
        for name in names:
            self._add_named(name)
        if white or ecorr:
            self._set_white(white, ecorr)

    # ------------------------------------------------------------------ layout building
    def _add_named(self, name):
        P = len(self.psrs)
        have = [p for p in self.psrs if name in p.signal_model]
        if not have:
            raise KeyError(f"no pulsar carries signal {name!r}")
        sm0 = have[0].signal_model[name]
        if "common" in name:
            f = np.asarray(sm0["f"], float)
            amp = np.sqrt(np.asarray(sm0["psd"], float) * _df(f))
            L = batch_factor(orf_matrix(self.psrs, sm0["orf"], sm0.get("hmap")))
            self.add_signal(name, 1, f, amp, idx=float(sm0["idx"]), L=L)
            return
        nm = max(len(p.signal_model[name]["f"]) for p in have)
        f = np.zeros((P, nm))
        amp = np.zeros((P, nm))
        mask = None
        for i, p in enumerate(self.psrs):
            if name in p.signal_model:
                sm = p.signal_model[name]
                fi = np.asarray(sm["f"], float)
                f[i, :len(fi)] = fi
                amp[i, :len(fi)] = np.sqrt(np.asarray(sm["psd"], float) * _df(fi))
                if len(fi) < nm:  # continue the grid with zero-amplitude modes
                    step = fi[0] if len(fi) else 1.0
                    f[i, len(fi):] = fi[-1] + step * np.arange(1, nm - len(fi) + 1)
            else:
                f[i] = np.arange(1, nm + 1) / max(np.ptp(p.toas), 1.0)
        idx = float(sm0["idx"])
        if "system_noise" in name:
            backend = name.split("system_noise_")[1]
            mask = np.concatenate([p.backend_flags == backend for p in self.psrs]).astype(np.uint8)
            idx = 0.0
        self.add_signal(name, 0, f, amp, idx=idx, mask=mask)

    def add_signal(self, name, kind, f, amp, idx=0.0, freqf=1400.0, L=None, mask=None):
        """Add one GP: kind 0 per-pulsar (f, amp [P, N]) or kind 1 common (f, amp [N], L [P, P])."""
        sid = self.ctx.batch_add_signal(kind, f, amp, idx=idx, freqf=freqf, L=L, mask=mask)
        self.segments.append(dict(name=name, kind=kind, f=np.asarray(f, float), amp=np.asarray(amp, float),
                                  idx=float(idx), freqf=float(freqf), L=L, mask=mask, id=sid))
        return sid

    def _set_white(self, white, ecorr):
        sigma = np.concatenate([p._white_sigma2() ** 0.5 for p in self.psrs]) if white else None
        blocks, esig = [], []
        if ecorr:
            for i, p in enumerate(self.psrs):
                for b in p.backends:
                    key = f"{p.name}_{b}_log10_ecorr"
                    if key not in p.noisedict:
                        continue
                    for q in p.ecorr_blocks(backends=[b]):
                        blocks.append(q + self.offs[i])
                        esig.append(10 ** p.noisedict[key])
        self.sigma = sigma
        self.blocks = blocks
        self.ecorr_sigma = np.array(esig)
        self.ctx.batch_set_white(sigma, blocks if blocks else None, self.ecorr_sigma if blocks else None)

    # ------------------------------------------------------------------ running
    @property
    def n_toa(self):
        return int(self.offs[-1])

    def synth(self, n_real, seed=0, real0=0, to_host=True, coeffs=False):
        """Realizations real0 .. real0+n_real-1: returns [n_real, n_toa] (host) or None (device only)."""
        return self.ctx.batch_synth(seed, real0, n_real, to_host=to_host, coeffs=coeffs)

    def synth_from_z(self, z):
        """Validation mode: z [n_real, n_seg, P, N_max, 2] standard normals (cos, sin)."""
        return self.ctx.batch_synth_from_z(z)

    def correlations(self, normalized=True):
        """Mean over the last block's realizations of the zero-lag cross-correlation matrix
        dot(res_a, res_b)/n (correlated_noises.py:14-19), normalized per realization by the
        auto-correlations if `normalized`. Computed on device; pulsars must share the TOA count."""
        _, _, R = self.ctx.batch_device_out()
        return self.ctx.batch_correlations(2 if normalized else 1) / R

    def hd_curve(self, bins=10, estimator="ratio"):
        """(mean, std, bin centres) of the pairwise correlations against angular separation
        (correlated_noises.py:21-47) for the last block. estimator "ratio": mean cross-power over
        sqrt(mean auto-powers) (consistent); "per_realization": mean of per-realization normalized
        correlations (biased toward 0 by O(1/n_eff) for red processes)."""
        if estimator == "ratio":
            C = self.correlations(normalized=False)
            d = np.sqrt(np.diag(C))
            C = C / np.outer(d, d)
        else:
            C = self.correlations(normalized=True)
        pos = np.array([p.pos for p in self.psrs])
        iu = np.triu_indices(len(self.psrs), 1)
        angles = np.arccos(np.clip(pos @ pos.T, -1.0, 1.0))[iu]
        return bin_curve(C[iu], angles, bins)

    def checksums(self):
        """Per-realization (sum, sum of squares) of the last block, computed on device."""
        return self.ctx.batch_checksums()

    def split(self, block):
        """[n_real, n_toa] -> list of per-pulsar [n_real, n_p] views."""
        return [block[..., self.offs[i]:self.offs[i + 1]] for i in range(len(self.psrs))]


def simulate_batch(psrs, n_real, seed=0, real0=0, signals=None, white=True, ecorr=False, device=None):
    """One-call convenience: [n_real, n_toa_total] residual realizations of the array's noise model."""
    return BatchSimulator(psrs, signals=signals, white=white, ecorr=ecorr, device=device).synth(
        n_real, seed=seed, real0=real0)
