"""SURVEY.md §8(d)(i) same-host cross-check of the CPU baseline (container-only: imports the read-only reference).

Times, on one core each and on the same C2 inputs (bench.py's array: 100 psr x 2000 TOAs, RN30 + DM100 + HD GWB30),
one re-drawn realization of
  * the reference itself: per pulsar add_red_noise / add_dm_noise with the pulsar's noisedict amplitudes (each
    subtracts the stored signal first, fake_pta.py:266-267), then add_common_correlated_noise (subtract, SVD per
    multivariate_normal call, per-mode passes; correlated_noises.py:133-160);
  * the oracle's restatement that bench.py's cpu_baseline leg runs on the GPU box (oracle.redraw_loop);
and writes their ratio to profiles/r03_cpu_crosscheck.json.

    OMP_NUM_THREADS=1 python tools/cpu_crosscheck.py [n_real]
"""
import os

for _k in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
    os.environ[_k] = "1"
import json  # noqa: E402
import platform  # noqa: E402
import sys  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
import ref_shim  # noqa: E402


def main():
    n_real = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    fp, cn, _ = ref_shim.load_reference()
    from oracle import fakepta_oracle as O
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=100, Tobs=10, ntoas=2000, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": 100, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3, components=30)
    # the restatement's inputs, taken from the reference's own objects
    P = len(psrs)
    segs = []
    for sig, idx in (("red_noise", 0.0), ("dm_gp", 2.0)):
        segs.append(dict(kind=0, f=np.array([p.signal_model[sig]["f"] for p in psrs]),
                         psd=np.array([p.signal_model[sig]["psd"] for p in psrs]), idx=idx))
    sm = psrs[0].signal_model["gw_common"]
    segs.append(dict(kind=1, f=np.asarray(sm["f"]), psd=np.asarray(sm["psd"]), idx=0.0, orf=cn.hd(psrs)))
    stored = {}
    for si, (sig, kind) in enumerate((("red_noise", 0), ("dm_gp", 0), ("gw_common", 1))):
        for p in range(P):
            stored[(si, p)] = np.array(psrs[p].signal_model[sig]["fourier"], dtype=float)
    res = [p.residuals.copy() for p in psrs]
    toas, freqs = [p.toas for p in psrs], [p.freqs for p in psrs]

    def ref_once():
        for p in psrs:
            nd = p.noisedict
            p.add_red_noise(spectrum="powerlaw", log10_A=nd[p.name + "_red_noise_log10_A"],
                            gamma=nd[p.name + "_red_noise_gamma"])
            p.add_dm_noise(spectrum="powerlaw", log10_A=nd[p.name + "_dm_gp_log10_A"],
                           gamma=nd[p.name + "_dm_gp_gamma"])
        cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3, components=30)

    rs = np.random.RandomState(7)
    t_ref, t_port = [], []
    for _ in range(n_real):  # interleaved, so drifts in the host's clock affect both alike
        t0 = time.perf_counter()
        ref_once()
        t_ref.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        O.redraw_loop(toas, freqs, segs, res, stored, rs)
        t_port.append(time.perf_counter() - t0)
    n_toa = sum(len(t) for t in toas)
    out = {
        "what": "one re-drawn C2 realization (100 psr x 2000 TOAs, RN30 + DM100 + HD GWB30), 1 thread each",
        "reference_s_per_realization": float(np.median(t_ref)), "reference_all_s": t_ref,
        "restatement_s_per_realization": float(np.median(t_port)), "restatement_all_s": t_port,
        "ratio_restatement_over_reference": float(np.median(t_port) / np.median(t_ref)),
        "reference_samples_per_s": n_toa / float(np.median(t_ref)),
        "restatement_samples_per_s": n_toa / float(np.median(t_port)),
        "restatement": "oracle/fakepta_oracle.py redraw_loop (bench.py cpu_baseline leg)",
        "reference": "/root/reference fakepta.fake_pta.Pulsar.add_red_noise / add_dm_noise, "
                     "fakepta.correlated_noises.add_common_correlated_noise (tools/ref_shim.py)",
        "host": platform.processor() or platform.machine(), "cpu_model": _cpu_model(),
        "numpy": np.__version__, "threads": 1,
    }
    path = os.path.join(ROOT, "profiles", "r03_cpu_crosscheck.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
