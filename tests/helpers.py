"""Shared helpers for the GPU parity tests: random array layouts and oracle conversion."""
import numpy as np

from oracle import fakepta_oracle as O


def variant_build(capi):
    """The loaded library is a variant build (make variant DEFS=-DFPTA_DIAG_KERNELS): it holds the diagnostic kernels
    and accepts the option values measured slower than the shipped ones, which the product library refuses."""
    return bool(capi.build_flags() & capi.BUILD_DIAG)


def assert_variant_refused(ctx, capi, key, value):
    """The product library refuses a variant-only option value and keeps the old one."""
    import pytest
    old = ctx.get_option(key)
    with pytest.raises(capi.FptaError, match="variant"):
        ctx.set_option(key, value)
    assert ctx.get_option(key) == old


def oracle_segments(sim):
    """BatchSimulator.segments -> oracle Segment list (same layout and semantics)."""
    return [O.Segment(s["kind"], (2.0 * np.pi) * s["f"], s["amp"], idx=s["idx"], freqf=s["freqf"], L=s["L"],
                      mask=s["mask"]) for s in sim.segments]


def random_layout(rng, P, n_range=(40, 300), t_max=3.2e8, ragged=True):
    if ragged:
        n = rng.integers(n_range[0], n_range[1], size=P)
    else:
        n = np.full(P, n_range[1])
    offs = np.concatenate([[0], np.cumsum(n)]).astype(np.int64)
    toas = np.concatenate([np.sort(rng.uniform(0.05 * t_max, t_max, k)) for k in n])
    nu = np.abs(rng.choice([1400.0, 800.0, 2500.0], size=offs[-1]) + rng.normal(0, 10, offs[-1]))
    return offs, toas, nu


def per_psr_signal(rng, offs, toas, n_modes, log10_A=-13.5, gamma=3.0):
    P = len(offs) - 1
    T = np.maximum([np.ptp(toas[offs[i]:offs[i + 1]]) for i in range(P)], 1e7)
    f = np.arange(1, n_modes + 1)[None, :] / T[:, None]
    df = np.diff(np.concatenate([np.zeros((P, 1)), f], axis=1), axis=1)
    la = rng.uniform(log10_A - 1, log10_A + 0.5, size=P)[:, None]
    amp = np.sqrt(O.powerlaw(f, la, gamma) * df)
    return f, amp


def common_signal(rng, offs, toas, n_modes, log10_A=-14.5, gamma=13 / 3, orf="hd", pos=None):
    P = len(offs) - 1
    f = np.arange(1, n_modes + 1) / np.ptp(toas)
    amp = np.sqrt(O.powerlaw(f, log10_A, gamma) * O.delta_f(f))
    if pos is None:
        v = rng.normal(size=(P, 3))
        pos = v / np.linalg.norm(v, axis=1)[:, None]
    L = O.mvn_factor(O.ORFS[orf](pos))
    return f, amp, L, pos


class EnterpriseStandin:
    """Stand-in for an enterprise.pulsar.Pulsar built from fixture G8's arrays (tools/gen_golden.py
    g8_standin_arrays): exactly the attributes copy_array reads (reference fake_pta.py:687-712)."""

    def __init__(self, a, i):
        lo, hi = a["offs"][i], a["offs"][i + 1]
        self.name = str(a["names"][i])
        self.toas = a["toas"][lo:hi].copy()
        self.freqs = a["freqs"][lo:hi].copy()
        self.toaerrs = a["toaerrs"][lo:hi].copy()
        self.backend_flags = a["backend_flags"][lo:hi].copy()
        self.residuals = np.zeros(hi - lo)
        self.theta, self.phi = float(a["theta"][i]), float(a["phi"][i])
        self.Mmat = np.stack([np.ones(hi - lo), self.toas - self.toas[0]], 1)
        self.fitpars = ["Offset", "F0"]
        self.pdist = (1.0, 0.2)
        self.planetssb = None
        self.pos_t = None


def g8_inputs(golden):
    """(stand-in pulsars, noisedict, custom_models, fixture arrays) of fixture G8 (examples/make_fake_array.py)."""
    g = golden("g8_example_workflow.npz")
    nd = golden("g8_noisedict_dr2_newsys_trim.json")
    cm = golden("g8_custom_models_newsys_trim.json")
    return [EnterpriseStandin(g, i) for i in range(len(g["names"]))], nd, cm, g
