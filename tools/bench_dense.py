"""Timings of the dense-covariance path on one GPU, next to the
reference-faithful numpy restatement (oracle) on the host.

    python tools/bench_dense.py [--sizes 2000 10000] [--real 1024] [--cpu]

Per size n (one pulsar, RN30 + DM100 + Sv30 = K 320 basis columns, white noise):
  cov     fpta_gp_covariance   basis + Gram (MFMA), n x n download included in the wall time
  wiener  fpta_noise_wiener    covariance + Cholesky + two substitutions
  draw    fpta_noise_draw      covariance + Cholesky + R draws (MFMA triangular product), download incl.
Device time per call from HIP events (kernel stats, FPTA_K_DENSE) and Gram / factor FLOP rates.
--cpu adds the oracle timings (reference formulation: basis loop, np.dot with np.diag, np.linalg.inv).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def case(n, seed=0):
    from oracle import fakepta_oracle as O
    rng = np.random.default_rng(seed)
    yr = 365.25 * 86400
    toas = np.sort(rng.uniform(0.0, 12 * yr, n)) + 53000 * 86400.0
    nu = rng.choice([800.0, 1400.0, 2100.0], n) + rng.normal(0, 5, n)
    T = toas.max() - toas.min()
    segs, osigs = [], []
    for nm, idx in ((30, 0.0), (100, 2.0), (30, 4.0)):
        f = np.arange(1, nm + 1) / T
        psd = O.powerlaw(f, rng.uniform(-14.5, -13.5), rng.uniform(1.5, 4.5))
        segs.append((f, psd * O.delta_f(f), idx, 1400.0))
        osigs.append((f, psd, idx))
    white = (3e-7 * rng.uniform(0.5, 2.0, n)) ** 2
    return toas, nu, segs, osigs, white


def timed(ctx, capi, fn, reps):
    fn()
    ctx.synchronize()
    ctx.set_option(capi.OPT_PROFILE, 1)
    ctx.reset_stats()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / reps
    dev = ctx.kernel_stats(capi.K_DENSE)[1] / reps * 1e-3
    ctx.set_option(capi.OPT_PROFILE, 0)
    return wall, dev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[2000, 10000])
    ap.add_argument("--real", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    from fakepta_amd import _capi as capi
    ctx = capi.get_context()
    for n in a.sizes:
        toas, nu, segs, osigs, white = case(n)
        K = 2 * sum(len(s[0]) for s in segs)
        r = np.random.default_rng(1).normal(size=n) * 1e-6
        w_cov, d_cov = timed(ctx, capi, lambda: ctx.gp_covariance(toas, nu, segs, white_var=white), a.reps)
        w_wie, d_wie = timed(ctx, capi, lambda: ctx.noise_wiener(toas, nu, segs, white, r), a.reps)
        R = a.real
        w_drw, d_drw = timed(ctx, capi, lambda: ctx.noise_draw(toas, nu, segs, white, 7, 0, R), a.reps)
        gram_flop = float(n) * n * K  # lower half of 2 n^2 K, mirrored
        chol_flop = n ** 3 / 3.0
        draw_flop = float(n) * n * R  # triangular: half of 2 n^2 R
        res = dict(path="dense", n_toa=n, K=K, realizations=R,
                   cov_wall_ms=w_cov * 1e3, cov_device_ms=d_cov * 1e3,
                   gram_tflops=gram_flop / d_cov / 1e12 if d_cov > 0 else None,
                   wiener_wall_ms=w_wie * 1e3, wiener_device_ms=d_wie * 1e3,
                   factor_plus_solve_ms=(d_wie - d_cov) * 1e3,
                   chol_tflops_est=chol_flop / max(d_wie - d_cov, 1e-9) / 1e12,
                   draw_wall_ms=w_drw * 1e3, draw_device_ms=d_drw * 1e3,
                   draw_samples_per_s=n * R / w_drw,
                   draw_samples_per_s_device=n * R / d_drw if d_drw > 0 else None,
                   draw_trmm_flop=draw_flop)
        if a.cpu and n <= 2000:
            from oracle import fakepta_oracle as O
            t0 = time.perf_counter()
            red = O.dense_cov(toas, nu, osigs)
            res["cpu_cov_s"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            O.wiener_reference(white, red, r)
            res["cpu_wiener_after_cov_s"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            np.random.multivariate_normal(np.zeros(n), red + np.diag(white))
            res["cpu_one_mvn_draw_s"] = time.perf_counter() - t0
            res["cpu_threads"] = os.environ.get("OMP_NUM_THREADS", "unset")
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
