"""Generate the committed golden fixtures under tests/golden/ (container-only).

Imports the read-only reference through tools/ref_shim.py and records its
inputs/outputs at small, seeded sizes. Run from the repo root:

    python tools/gen_golden.py

Never run on the GPU box (the reference is not there); the tests only read the
.npz/.json files this writes. Everything stored is data: inputs (TOAs, radio
frequencies, random draws in the reference's own draw order) and outputs
(PSDs, Fourier coefficients, residuals, ORF matrices, names, noisedicts).

Fixture map:
  g1_psd.npz          all six PSDs of fakepta/spectrum.py:12-86 on 3 grids x 3 parameter sets
  g2_single_psr.npz   one ragged 2-backend pulsar: RN30 / DM100 (idx 2) / Sv30 (idx 4),
                      replace-on-reinject, backend-masked injection, white noise,
                      reconstruct_signal, quantise_ecorr
  g3_common.npz       25-pulsar Fibonacci array: common GP with hd / monopole / dipole / curn
  g4_make_fake_array.npz + g4_noisedict.json
                      config 1 (BASELINE configs[0]) end-to-end with np.random.seed(0)
  g5_tutorial.json    known answers printed in examples/tutorial.ipynb
  g6_dense_cov.npz    one 2-backend pulsar: make_time_correlated_noise_cov per GP,
                      make_noise_covariance_matrix, draw_noise_model(residuals) (Wiener)
  g7_ref_pulsars.pkl  4 Pulsar objects pickled by the reference (class fakepta.fake_pta.Pulsar)
  g7_ref_pulsars.npz  the reference's reconstruct_signal() on them, then its residuals after
                      np.random.seed(32) + add_red_noise (replace) + add_common_correlated_noise
  g8_example_workflow.npz + g8_example_workflow.json
                      examples/make_fake_array.py:31-47 with the reference's own shipped
                      examples/simulated_data/{noisedict,custom_models}_*newsys_trim.json (copied here as
                      data: g8_noisedict_dr2_newsys_trim.json, g8_custom_models_newsys_trim.json): copy_array
                      of 26 stand-in multi-backend EPTA pulsars (the example's pickle is a private file),
                      then make_ideal / add_white_noise / add_red_noise() / add_dm_noise() /
                      add_chromatic_noise() with no kwargs (noisedict-driven), then the HD GWB
  g9_common_components.npz
                      add_common_correlated_noise with len(f_psd) != components
                      (correlated_noises.py:142-160): 40 frequencies, components=30 (30 modes injected,
                      psd/f stored with 40 entries); and 20 frequencies, components=30 (IndexError after
                      the first 20 modes and one more draw pair)

Run a subset with  python tools/gen_golden.py g8 g9
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import ref_shim  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _ragged_epochs(rng, n, t0, cadence, keep_prob=0.75):
    keep = rng.random(n) < keep_prob
    return t0 + np.arange(1, n + 1)[keep] * cadence


def gen_g1(sp):
    yr = 365.25 * 24 * 3600
    grids = [np.arange(1, 31) / (10 * yr), np.arange(1, 101) / (15.3 * yr),
             np.geomspace(1e-9, 1e-7, 17)]
    out = {}
    params = {
        "powerlaw": [dict(log10_A=-14.0, gamma=3.0), dict(log10_A=-15.0, gamma=13 / 3),
                     dict(log10_A=-13.2, gamma=1.7)],
        "turnover": [dict(), dict(log10_A=-14.5, gamma=4.0, lf0=-8.2, kappa=2.0, beta=0.8),
                     dict(log10_A=-15.5, gamma=5.0, lf0=-8.9, kappa=10 / 3, beta=0.5)],
        "t_process": [dict(), dict(log10_A=-14.0, gamma=3.0), dict(log10_A=-14.0, gamma=3.0, alphas="ramp")],
        "t_process_adapt": [dict(), dict(log10_A=-14.0, gamma=3.0, alphas_adapt=2.5, nfreq=3.2),
                            dict(log10_A=-14.0, gamma=3.0, alphas_adapt="ramp")],
        "turnover_knee": [dict(log10_A=-15.0, gamma=13 / 3, lfb=-8.5, lfk=-7.5, kappa=10 / 3, delta=-1.0),
                          dict(log10_A=-14.0, gamma=4.0, lfb=-8.8, lfk=-7.9, kappa=2.0, delta=-0.5),
                          dict(log10_A=-14.7, gamma=3.0, lfb=-9.0, lfk=-8.0, kappa=1.0, delta=0.0)],
        "broken_powerlaw": [dict(log10_A=-15.0, gamma=13 / 3, delta=0.0, log10_fb=-8.5),
                            dict(log10_A=-14.0, gamma=4.0, delta=1.0, log10_fb=-8.0, kappa=0.3),
                            dict(log10_A=-14.5, gamma=3.0, delta=2.0, log10_fb=-7.8, kappa=0.1)],
    }
    meta = {}
    for name, plist in params.items():
        fn = getattr(sp, name)
        for gi, f in enumerate(grids):
            for pi, p in enumerate(plist):
                p = dict(p)
                for key in ("alphas", "alphas_adapt"):
                    if p.get(key) == "ramp":
                        p[key] = np.linspace(0.5, 2.0, len(f))
                key = f"{name}__g{gi}__p{pi}"
                out[key] = fn(f.copy(), **p)
                meta[key] = {k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in p.items()}
    for gi, f in enumerate(grids):
        out[f"grid{gi}"] = f
    out["meta_json"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, "g1_psd.npz"), **out)


def _draw_record(fn, n_draws):
    """Run fn(), and return the standard normals it consumed (legacy RandomState order)."""
    st = np.random.get_state()
    fn()
    st_after = np.random.get_state()
    np.random.set_state(st)
    z = np.random.standard_normal(n_draws)
    np.random.set_state(st_after)
    return z


def gen_g2(fp):
    rng = np.random.default_rng(7)
    yr = 365.25 * 24 * 3600
    epochs = _ragged_epochs(rng, 330, 0.35 * yr, 12.3 * 24 * 3600)
    np.random.seed(11)
    psr = fp.Pulsar(epochs, 3e-7, 1.1, 4.2, pdist=(1.0, 0.2), freqs=[1400],
                    backends=["A.1400", "B.800"],
                    custom_model={"RN": 30, "DM": 100, "Sv": 30})
    d = dict(toas=psr.toas.copy(), freqs=psr.freqs.copy(), Tspan=psr.Tspan,
             backend_flags=psr.backend_flags.astype("U"), name=np.array(psr.name))
    # noise parameters
    for b in psr.backends:
        psr.noisedict[f"{psr.name}_{b}_efac"] = {"A.1400": 1.3, "B.800": 0.8}[b]
        psr.noisedict[f"{psr.name}_{b}_log10_tnequad"] = {"A.1400": -6.5, "B.800": -7.2}[b]

    def inject(label, call, n_modes):
        before = psr.residuals.copy()
        z = _draw_record(call, 2 * n_modes)
        d[f"{label}_z"] = z
        d[f"{label}_delta"] = psr.residuals - before

    inject("rn", lambda: psr.add_red_noise(spectrum="powerlaw", log10_A=-13.4, gamma=3.3), 30)
    inject("dm", lambda: psr.add_dm_noise(spectrum="powerlaw", log10_A=-13.1, gamma=2.5), 100)
    inject("sv", lambda: psr.add_chromatic_noise(spectrum="powerlaw", log10_A=-13.6, gamma=2.0), 30)
    for sig, lab in (("red_noise", "rn"), ("dm_gp", "dm"), ("chrom_gp", "sv")):
        sm = psr.signal_model[sig]
        d[f"{lab}_f"] = sm["f"]
        d[f"{lab}_psd"] = sm["psd"]
        d[f"{lab}_fourier"] = sm["fourier"]
        d[f"{lab}_idx"] = float(sm["idx"])
        d[f"{lab}_reconstruct"] = psr.reconstruct_signal([sig])
    d["total_after_gp"] = psr.residuals.copy()
    d["reconstruct_all"] = psr.reconstruct_signal()
    # replace-on-reinject (fake_pta.py:266-267)
    before = psr.residuals.copy()
    z = _draw_record(lambda: psr.add_red_noise(spectrum="powerlaw", log10_A=-13.0, gamma=4.1), 60)
    d["rn2_z"] = z
    d["rn2_fourier"] = psr.signal_model["red_noise"]["fourier"]
    d["rn2_psd"] = psr.signal_model["red_noise"]["psd"]
    d["rn2_residuals"] = psr.residuals.copy()
    d["rn2_before"] = before
    # backend-masked injection (fake_pta.py:357-368) is NOT recorded: the reference raises
    # "operands could not be broadcast" whenever the mask is partial, because
    # (freqf/self.freqs)**idx at :386 is full-length (defect D9). Parity unpinned.
    # white noise (fake_pta.py:201-230), no ECORR
    before = psr.residuals.copy()
    z = _draw_record(lambda: psr.add_white_noise(), len(psr.toas))
    d["wn_z"] = z
    d["wn_delta"] = psr.residuals - before
    d["wn_efac"] = np.array([psr.noisedict[f"{psr.name}_{b}_efac"] for b in ("A.1400", "B.800")])
    d["wn_tnequad"] = np.array([psr.noisedict[f"{psr.name}_{b}_log10_tnequad"] for b in ("A.1400", "B.800")])
    d["toaerrs"] = psr.toaerrs.copy()
    # quantise_ecorr on sub-day epochs (fake_pta.py:232-253, defect D2 preserved)
    ep = np.sort(np.concatenate([epochs[:40], epochs[:40] + 3600.0, epochs[5:9] + 7200.0]))
    np.random.seed(3)
    psr_q = fp.Pulsar(ep, 1e-6, 0.7, 1.0, backends=["A.1400", "B.800"],
                      custom_model={"RN": None, "DM": None, "Sv": None})
    q = psr_q.quantise_ecorr()
    d["q_toas"] = psr_q.toas
    d["q_flags"] = psr_q.backend_flags.astype("U")
    d["q_lens"] = np.array([len(b) for b in q])
    d["q_idx"] = np.concatenate(q) if q else np.zeros(0, int)
    np.savez_compressed(os.path.join(OUT, "g2_single_psr.npz"), **d)


def gen_g3(fp, cn):
    np.random.seed(5)
    psrs = fp.make_fake_array(npsrs=25, Tobs=None, ntoas=120, gaps=True, toaerr=1e-7, isotropic=True,
                              backends=["A.1400", "B.800"],
                              custom_model={"RN": None, "DM": None, "Sv": None})
    offs = np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])])
    d = dict(offs=offs, toas=np.concatenate([p.toas for p in psrs]),
             freqs=np.concatenate([p.freqs for p in psrs]),
             pos=np.array([p.pos for p in psrs]))
    N = 30
    for orf in ("hd", "monopole", "dipole", "curn"):
        for p in psrs:
            p.make_ideal()
        gam = {"hd": cn.hd, "monopole": cn.monopole, "dipole": cn.dipole, "curn": cn.curn}[orf](psrs)
        u, s, vt = np.linalg.svd(gam)
        d[f"{orf}_orf"] = gam
        d[f"{orf}_svdM"] = np.sqrt(s)[:, None] * vt
        idx = 2.0 if orf == "dipole" else 0
        z = _draw_record(lambda: cn.add_common_correlated_noise(psrs, orf=orf, spectrum="powerlaw", name="gw",
                                                                idx=idx, components=N,
                                                                log10_A=-14.2, gamma=13 / 3),
                         2 * N * len(psrs))
        d[f"{orf}_z"] = z.reshape(N, 2, len(psrs))  # per mode: sin draw first, then cos
        d[f"{orf}_idx"] = float(idx)
        d[f"{orf}_fourier"] = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
        d[f"{orf}_f"] = psrs[0].signal_model["gw_common"]["f"]
        d[f"{orf}_psd"] = psrs[0].signal_model["gw_common"]["psd"]
        d[f"{orf}_residuals"] = np.concatenate([p.residuals for p in psrs])
        d[f"{orf}_reconstruct"] = np.concatenate([p.reconstruct_signal(["gw_common"]) for p in psrs])
    np.savez_compressed(os.path.join(OUT, "g3_common.npz"), **d)


def gen_g4(fp):
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=25, Tobs=10, ntoas=1000, isotropic=True, gaps=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": None, "Sv": None})
    d = dict(offs=np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])]),
             toas=np.concatenate([p.toas for p in psrs]),
             freqs=np.concatenate([p.freqs for p in psrs]),
             residuals=np.concatenate([p.residuals for p in psrs]),
             names=np.array([p.name for p in psrs]),
             pos=np.array([p.pos for p in psrs]),
             rn_fourier=np.array([p.signal_model["red_noise"]["fourier"] for p in psrs]),
             rn_psd=np.array([p.signal_model["red_noise"]["psd"] for p in psrs]),
             rn_f=np.array([p.signal_model["red_noise"]["f"] for p in psrs]),
             Mmat0=psrs[0].Mmat, tm_F0=np.array([p.tm_pars["F0"][0] for p in psrs]))
    np.savez_compressed(os.path.join(OUT, "g4_make_fake_array.npz"), **d)
    nd = {}
    for p in psrs:
        nd.update({k: float(v) for k, v in p.noisedict.items()})
    with open(os.path.join(OUT, "g4_noisedict.json"), "w") as fh:
        json.dump(nd, fh, indent=0, sort_keys=True)
    # second end-to-end case: default custom_model (RN30 + DM100), two backends, random Tobs/ntoas
    np.random.seed(1)
    psrs = fp.make_fake_array(npsrs=6, Tobs=None, ntoas=None, gaps=True, toaerr=None,
                              backends=["A.1400", "B.800"], isotropic=False)
    d = dict(offs=np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])]),
             toas=np.concatenate([p.toas for p in psrs]),
             freqs=np.concatenate([p.freqs for p in psrs]),
             residuals=np.concatenate([p.residuals for p in psrs]),
             names=np.array([p.name for p in psrs]))
    np.savez_compressed(os.path.join(OUT, "g4b_make_fake_array.npz"), **d)


def gen_g5():
    nb = json.load(open("/root/reference/examples/tutorial.ipynb"))
    names = []
    psd = None
    for c in nb["cells"]:
        for o in c.get("outputs", []):
            txt = "".join(o.get("text", []))
            for line in txt.splitlines():
                if line.startswith("Creating psr "):
                    names.append(line.split()[-1])
            data = o.get("data", {}).get("text/plain")
            if data and "'psd': array(" in "".join(data):
                s = "".join(data)
                body = s.split("'psd': array([")[1].split("])")[0]
                psd = [float(x) for x in body.replace("\n", " ").split(",") if x.strip()]
    with open(os.path.join(OUT, "g5_tutorial.json"), "w") as fh:
        json.dump({"names_npsrs25_isotropic": names,
                   "rn_psd_log10A_m14_gamma3_30modes_Tobs10": psd,
                   "rn_f_first": 3.17834381e-09,
                   "source": "examples/tutorial.ipynb cell 5 output (names), cell 18 output (psd)"},
                  fh, indent=1)


def gen_g6(fp):
    rng = np.random.default_rng(17)
    yr = 365.25 * 24 * 3600
    epochs = _ragged_epochs(rng, 80, 0.2 * yr, 30.1 * 24 * 3600)
    np.random.seed(23)
    psr = fp.Pulsar(epochs, 2e-7, 0.4, 2.2, pdist=(1.0, 0.2), freqs=[1400],
                    backends=["A.1400", "B.800"],
                    custom_model={"RN": 30, "DM": 100, "Sv": 30})
    for b in psr.backends:
        psr.noisedict[f"{psr.name}_{b}_efac"] = {"A.1400": 1.2, "B.800": 0.9}[b]
        psr.noisedict[f"{psr.name}_{b}_log10_tnequad"] = {"A.1400": -6.8, "B.800": -7.1}[b]
    psr.add_red_noise(spectrum="powerlaw", log10_A=-13.9, gamma=3.1)
    psr.add_dm_noise(spectrum="powerlaw", log10_A=-13.5, gamma=2.2)
    psr.add_chromatic_noise(spectrum="powerlaw", log10_A=-13.8, gamma=1.8)
    psr.add_white_noise()
    d = dict(toas=psr.toas.copy(), freqs=psr.freqs.copy(), toaerrs=psr.toaerrs.copy(),
             backend_flags=psr.backend_flags.astype("U"), name=np.array(psr.name),
             residuals=psr.residuals.copy(),
             efac=np.array([psr.noisedict[f"{psr.name}_{b}_efac"] for b in ("A.1400", "B.800")]),
             tnequad=np.array([psr.noisedict[f"{psr.name}_{b}_log10_tnequad"] for b in ("A.1400", "B.800")]))
    for sig, lab in (("red_noise", "rn"), ("dm_gp", "dm"), ("chrom_gp", "sv")):
        sm = psr.signal_model[sig]
        d[f"{lab}_f"] = sm["f"]
        d[f"{lab}_psd"] = sm["psd"]
        d[f"{lab}_idx"] = float(sm["idx"])
        d[f"{lab}_cov"] = psr.make_time_correlated_noise_cov(signal=sig)
    white_cov, red_cov = psr.make_noise_covariance_matrix()
    d["white_cov"] = white_cov
    d["red_cov"] = red_cov
    d["wiener"] = psr.draw_noise_model(residuals=psr.residuals)
    np.savez_compressed(os.path.join(OUT, "g6_dense_cov.npz"), **d)


def gen_g7(fp, cn):
    """Pulsar objects pickled by the reference itself (class path fakepta.fake_pta.Pulsar, the way
    examples/make_fake_array.py:65 saves an array) and what the reference computes on them afterwards:
    the drop-in must unpickle them and continue the session with the same results."""
    import pickle
    np.random.seed(31)
    psrs = fp.make_fake_array(npsrs=4, Tobs=5, ntoas=150, gaps=True, toaerr=1e-7, isotropic=True,
                              backends=["A.1400", "B.800"], custom_model={"RN": 20, "DM": 25, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", components=15, log10_A=-14.3, gamma=13 / 3)
    assert type(psrs[0]).__module__ == "fakepta.fake_pta"
    with open(os.path.join(OUT, "g7_ref_pulsars.pkl"), "wb") as fh:
        pickle.dump(psrs, fh, protocol=4)
    d = {}
    for i, p in enumerate(psrs):
        d[f"residuals_{i}"] = p.residuals.copy()
        d[f"reconstruct_all_{i}"] = p.reconstruct_signal()
    np.random.seed(32)
    for p in psrs:
        p.add_red_noise(spectrum="powerlaw", log10_A=-13.5, gamma=3.5)  # replace-on-reinject
    cn.add_common_correlated_noise(psrs, orf="hd", components=15, log10_A=-14.0, gamma=4.0)
    for i, p in enumerate(psrs):
        d[f"residuals_after_{i}"] = p.residuals.copy()
        d[f"rn_fourier_after_{i}"] = p.signal_model["red_noise"]["fourier"].copy()
    np.savez_compressed(os.path.join(OUT, "g7_ref_pulsars.npz"), **d)


G8_ND = "g8_noisedict_dr2_newsys_trim.json"
G8_CM = "g8_custom_models_newsys_trim.json"


def g8_standin_arrays(noisedict, names, seed=2024):
    """Inputs of the stand-in ENTERPRISE pulsars: per pulsar the backends its noisedict names (EPTA
    multi-backend flags, e.g. 'EFF.P217.1380'), ragged per-backend observing campaigns on real-MJD epochs
    (seconds), 1-2 sub-band TOAs per epoch at the flag's frequency +- 64 MHz, TOA errors 10^U(-7,-5.5), and
    the sky position read from the J-name. Returns flat arrays + CSR offsets (all data, no objects)."""
    rng = np.random.default_rng(seed)
    day = 86400.0
    toas, freqs, errs, flags, offs, theta, phi = [], [], [], [], [0], [], []
    for name in names:
        bks = sorted({k[len(name) + 1:-len("_efac")] for k in noisedict
                      if k.startswith(name + "_") and k.endswith("_efac")})
        sgn = 1.0 if name[5] == "+" else -1.0
        dec = sgn * (int(name[6:8]) + int(name[8:10]) / 60.0)
        theta.append(np.pi / 2 - np.pi / 180.0 * dec)
        phi.append(2 * np.pi * (int(name[1:3]) + int(name[3:5]) / 60.0) / 24.0)
        t, f, b = [], [], []
        for bk in bks:
            start = rng.uniform(50500.0, 56500.0)
            end = min(59500.0, start + rng.uniform(900.0, 3000.0))
            ep = np.arange(start, end, rng.uniform(25.0, 60.0))
            ep = ep[rng.random(len(ep)) < 0.8]
            ep = ep + rng.normal(0.0, 1.0, size=len(ep))
            nsub = int(rng.integers(1, 3))
            nominal = float(bk.split(".")[-1])
            for j in range(nsub):
                t.append(ep * day + 900.0 * j)
                f.append(nominal + (0.0 if nsub == 1 else (-64.0 if j == 0 else 64.0)) + np.zeros(len(ep)))
                b += [bk] * len(ep)
        t = np.concatenate(t)
        order = np.argsort(t, kind="stable")
        toas.append(t[order])
        freqs.append(np.concatenate(f)[order])
        flags += list(np.array(b)[order])
        errs.append(10 ** rng.uniform(-7.0, -5.5, size=len(t)))
        offs.append(offs[-1] + len(t))
    return dict(names=np.array(names), offs=np.array(offs, dtype=np.int64), toas=np.concatenate(toas),
                freqs=np.concatenate(freqs), toaerrs=np.concatenate(errs), backend_flags=np.array(flags),
                theta=np.array(theta), phi=np.array(phi))


class _EnterprisePulsar:
    """Stand-in for an enterprise.pulsar.Pulsar: exactly the attributes copy_array reads
    (fake_pta.py:687-712)."""

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


def gen_g8(fp, cn):
    import shutil
    ex = os.path.join(ref_shim.REF, "examples", "simulated_data")
    shutil.copyfile(os.path.join(ex, "noisedict_dr2_newsys_trim.json"), os.path.join(OUT, G8_ND))
    shutil.copyfile(os.path.join(ex, "custom_models_newsys_trim.json"), os.path.join(OUT, G8_CM))
    noisedict = json.load(open(os.path.join(OUT, G8_ND)))
    custom_models = json.load(open(os.path.join(OUT, G8_CM)))
    names = sorted(custom_models)
    a = g8_standin_arrays(noisedict, names)
    psrs_0 = [_EnterprisePulsar(a, i) for i in range(len(names))]
    np.random.seed(8)
    psrs = fp.copy_array(psrs_0, noisedict, custom_models)            # examples/make_fake_array.py:34
    d = dict(a)
    d["seed"] = np.array(8)
    for p in psrs:                                                     # :37-43
        p.make_ideal()
        p.add_white_noise()
        p.add_red_noise()
        p.add_dm_noise()
        p.add_chromatic_noise()
    d["residuals_noise"] = np.concatenate([p.residuals for p in psrs])
    cn.add_common_correlated_noise(psrs, log10_A=-15., gamma=13 / 3, orf="hd")   # :47
    d["residuals"] = np.concatenate([p.residuals for p in psrs])
    d["copied_freqs"] = np.concatenate([p.freqs for p in psrs])
    models = {}
    for i, p in enumerate(psrs):
        models[p.name] = {}
        for sig, sm in p.signal_model.items():
            key = f"{i}_{sig}"
            d[key + "_f"] = np.asarray(sm["f"], float)
            d[key + "_psd"] = np.asarray(sm["psd"], float)
            d[key + "_fourier"] = np.asarray(sm["fourier"], float)
            d[key + "_reconstruct"] = p.reconstruct_signal([sig])
            models[p.name][sig] = {"nbin": int(sm["nbin"]), "idx": float(sm["idx"]), "spectrum": sm["spectrum"]}
    np.savez_compressed(os.path.join(OUT, "g8_example_workflow.npz"), **d)
    with open(os.path.join(OUT, "g8_example_workflow.json"), "w") as fh:
        json.dump({"noisedicts": {p.name: {k: float(v) for k, v in p.noisedict.items()} for p in psrs},
                   "signal_models": models, "Tspan": {p.name: float(p.Tspan) for p in psrs},
                   "source": "examples/make_fake_array.py:31-47 via tools/gen_golden.py gen_g8"},
                  fh, indent=0, sort_keys=True)


def gen_g9(fp, cn):
    """add_common_correlated_noise when len(f_psd) != components (correlated_noises.py:118-160)."""
    np.random.seed(9)
    psrs = fp.make_fake_array(npsrs=8, Tobs=8, ntoas=90, gaps=True, toaerr=1e-7, isotropic=True,
                              backends=["A.1400", "B.800"], custom_model={"RN": None, "DM": None, "Sv": None})
    tspan = max(p.toas.max() for p in psrs) - min(p.toas.min() for p in psrs)
    d = dict(offs=np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])]),
             toas=np.concatenate([p.toas for p in psrs]), freqs=np.concatenate([p.freqs for p in psrs]))
    d["pos"] = np.array([p.pos for p in psrs])
    P = len(psrs)
    f40 = np.arange(1, 41) / tspan
    for p in psrs:
        p.make_ideal()
    z = _draw_record(lambda: cn.add_common_correlated_noise(psrs, orf="hd", components=30, f_psd=f40, log10_A=-14.5,
                                                            gamma=13 / 3, idx=2), 2 * 30 * P)
    d["long_z"] = z.reshape(30, 2, P)
    sm = psrs[0].signal_model["gw_common"]
    d["long_f"], d["long_psd"], d["long_nbin"] = sm["f"], sm["psd"], np.array(sm["nbin"])
    d["long_fourier"] = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
    d["long_residuals"] = np.concatenate([p.residuals for p in psrs])
    d["long_reconstruct"] = np.concatenate([p.reconstruct_signal(["gw_common"]) for p in psrs])
    d["long_next_draw"] = np.random.standard_normal(4)
    np.random.seed(19)
    for p in psrs:
        p.make_ideal()
    f20 = np.arange(1, 21) / tspan
    st = np.random.get_state()
    try:
        cn.add_common_correlated_noise(psrs, orf="hd", components=30, f_psd=f20, log10_A=-14.5, gamma=13 / 3)
        raise AssertionError("reference accepted len(f_psd) < components")
    except IndexError as e:
        d["short_error"] = np.array(str(e))
    st_after = np.random.get_state()
    np.random.set_state(st)
    d["short_z"] = np.random.standard_normal(2 * 21 * P).reshape(21, 2, P)
    np.random.set_state(st_after)
    d["short_residuals"] = np.concatenate([p.residuals for p in psrs])
    d["short_fourier"] = np.array([p.signal_model["gw_common"]["fourier"] for p in psrs])
    d["short_next_draw"] = np.random.standard_normal(4)
    np.savez_compressed(os.path.join(OUT, "g9_common_components.npz"), **d)


def main():
    os.makedirs(OUT, exist_ok=True)
    fp, cn, sp = ref_shim.load_reference()
    which = set(sys.argv[1:]) or {"g1", "g2", "g3", "g4", "g5", "g6", "g7", "g8", "g9"}
    for key, fn in (("g1", lambda: gen_g1(sp)), ("g2", lambda: gen_g2(fp)), ("g3", lambda: gen_g3(fp, cn)),
                    ("g4", lambda: gen_g4(fp)), ("g5", gen_g5), ("g6", lambda: gen_g6(fp)),
                    ("g7", lambda: gen_g7(fp, cn)), ("g8", lambda: gen_g8(fp, cn)), ("g9", lambda: gen_g9(fp, cn))):
        if key in which:
            fn()
    for fn in sorted(os.listdir(OUT)):
        print(fn, os.path.getsize(os.path.join(OUT, fn)))


if __name__ == "__main__":
    main()
