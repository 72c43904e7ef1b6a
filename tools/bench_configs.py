"""Timings of the BASELINE configs other than the driver's headline (bench.py = C2), one GPU.

    python tools/bench_configs.py [c1] [c3] [c4] [c5] [--c3-real 100000] [--opt NAME=VALUE ...]

c1  make_fake_array(25 psr, Tobs 10, ntoas 1000, gaps, RN30) drop-in latency, seed 0
    (the reference: 0.045 s on the survey container's CPU)
c3  100-psr HD GWB30 only (K = 60), realizations streamed in batches of 7168 (bench.py --c3-batch), checksums only
c4  1000 psr x 10k TOAs, HD GWB100 (K = 200), 1000x1000 ORF factor, R = 256
c5  100 psr, RN30 + DM100 + Sv100 + HD30 + monopole30 + dipole30 + white + ECORR (K = 640), R = 1024
Prints one JSON line per config: samples/s end-to-end (pipelined, no per-kernel events) and per-kernel-class
HIP-event times of a one-stream rerun (isolated launch durations; the rocprofv3 statistics under profiles/ are the
per-kernel record).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


OPTS = []  # --opt NAME=VALUE: library options set on every context a config creates (A/B runs)


def new_context(capi):
    ctx = capi.Context(0)
    for kv in OPTS:
        name, val = kv.split("=")
        ctx.set_option(getattr(capi, "OPT_" + name.upper()), int(val))
    return ctx


def kernel_times(ctx, capi, steps):
    return {n: ctx.kernel_stats(k)[1] / steps for n, k in
            (("gen", capi.K_GEN), ("mix", capi.K_MIX), ("grid", capi.K_GRID), ("synth", capi.K_SYNTH),
             ("white", capi.K_WHITE))}


def timed(ctx, capi, fn, steps, warmup=2):
    """Wall time of `steps` calls of fn (the shipped pipelined configuration, no per-kernel events)."""
    for _ in range(warmup):
        fn(0)
    ctx.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        fn(s + warmup)
    ctx.synchronize()
    return time.perf_counter() - t0


def isolated(ctx, capi, fn, steps, first=1000):
    """Per-kernel-class HIP-event times per step with ONE stream (FPTA_OPT_OVERLAP 0), after the timed run: the
    launches are serial there, so the intervals are launch durations (in the pipelined run they overlap and are
    not). The judged per-kernel figures are the rocprofv3 kernel statistics under profiles/."""
    ctx.set_option(capi.OPT_OVERLAP, 0)
    try:
        fn(first)
        ctx.synchronize()
        ctx.set_option(capi.OPT_PROFILE, 1)
        ctx.reset_stats()
        for s in range(steps):
            fn(first + 1 + s)
        ctx.synchronize()
        return kernel_times(ctx, capi, steps)
    finally:
        ctx.set_option(capi.OPT_PROFILE, 0)
        ctx.set_option(capi.OPT_OVERLAP, 1)


def c1():
    from fakepta import fake_pta as fp
    kw = dict(npsrs=25, Tobs=10, ntoas=1000, isotropic=True, gaps=True, toaerr=1e-7, backends="NUPPI.1400",
              custom_model={"RN": 30, "DM": None, "Sv": None})
    np.random.seed(0)
    fp.make_fake_array(**kw)  # warm (context creation, code objects)
    ts = []
    for _ in range(5):
        np.random.seed(0)
        t0 = time.perf_counter()
        psrs = fp.make_fake_array(**kw)
        ts.append(time.perf_counter() - t0)
    n = sum(len(p.toas) for p in psrs)
    return dict(config="c1", n_toa=n, latency_s_median=float(np.median(ts)), latency_s_min=float(min(ts)),
                samples_per_s=n / float(np.median(ts)), reference_cpu_s=0.045,
                note="drop-in path: host np.random draws + one GPU call per injection; latency-bound")


HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def _interp_entry(gi, n_toa, R, ms, K=None, traffic_R=None):
    """The interpolation kernel of a config's last block (the dominant kernel) and its HBM fraction: 8 B per residual
    sample written over its isolated (one-stream) launch time; with the newest matching PMC record
    under profiles/ (tools/gpu_evidence6.sh: FETCH_SIZE doubled + WRITE_SIZE of the same kernel and shape), its HBM
    bytes per launch over the algorithmic bytes."""
    gbs = 8.0 * n_toa * R / (ms / 1e3) / 1e9 if ms else None
    entry = dict(kernel=gi["interp_kernel"], avg_launch_ms=ms, algorithmic_bytes=8.0 * n_toa * R, achieved_GBps=gbs,
                 frac=gbs / HBM_PEAK_GBS if gbs else None)
    if K is not None and gi["interp_kernel"]:
        import bench
        RR = traffic_R or R
        traffic, src = bench.pmc_traffic(gi["interp_kernel"], {"K": K, "n_toa": n_toa}, RR, None)
        entry.update(traffic_bytes=traffic, traffic_source=src,
                     traffic_over_algorithmic=traffic / (8.0 * n_toa * RR) if traffic else None)
    return entry


def c3_job(total=100000, batch=7168, jobs=2):
    """C3 as bench.py --config c3 runs it on one GPU: the HD GWB job of `total` realizations streamed through
    simulate_sharded (fused partial checksums, pipelined batches), `jobs` timed jobs after one warm job; the
    fused-checksum interpolation's average launch time over the timed jobs (HIP events; it co-runs with the next
    batch's draws and DFT)."""
    import bench
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator, simulate_sharded
    ctx = new_context(_capi)
    psrs = bench.build_array(100, 2000, "c3")
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    info = ctx.batch_info()
    simulate_sharded(sim, total, seed=1234, real0=0, batch=batch)
    ctx.synchronize()
    ctx.set_option(_capi.OPT_PROFILE, 1)
    ctx.reset_stats()
    t0 = time.perf_counter()
    for j in range(jobs):
        sums = simulate_sharded(sim, total, seed=1234, real0=(j + 1) * total, batch=batch)
    ctx.synchronize()
    dt = (time.perf_counter() - t0) / jobs
    n, ms = ctx.kernel_stats(_capi.K_SYNTH)
    ctx.set_option(_capi.OPT_PROFILE, 0)
    gi = ctx.batch_grid_info()
    ctx.close()
    n_batches = -(-total // batch)
    entry = _interp_entry(gi, info["n_toa"], total / n_batches, ms / max(n, 1), K=info["K"], traffic_R=batch)
    entry["note"] = "average over the job's batches (the short last one included), pipelined (HIP events)"
    return dict(job_ms=dt * 1e3, samples_per_s=info["n_toa"] * total / dt, realizations=total, batch=batch,
                checksum=float(np.sum(sums[:, 1])), interp=entry)


def sub_records():
    """Compact C3 / C5 / C4 (per-GPU share) records for bench.py's line, each on a fresh context after bench.py's
    timed C2 region (they never change its value). A config that fails records its error instead."""
    out = {}
    for key, fn in (("c3", c3_job), ("c5", lambda: c5(steps=10)), ("c4_per_gpu", lambda: c4(steps=5))):
        t0 = time.perf_counter()
        try:
            r = fn()
            out[key] = {k: r[k] for k in ("job_ms", "ms_per_step", "samples_per_s", "realizations", "interp",
                                          "mix_ms_isolated", "checksum") if k in r}
        except Exception as e:  # recorded, not fatal: the headline line must still print
            out[key] = {"error": repr(e)}
        out[key]["wall_s"] = time.perf_counter() - t0
    return out


def fib(P):
    i = np.arange(P) + 0.5
    th = np.arccos(1 - 2 * i / P)
    ph = np.mod(2 * np.pi * i / ((1 + 5 ** 0.5) / 2), 2 * np.pi)
    return np.stack([np.cos(ph) * np.sin(th), np.sin(ph) * np.sin(th), np.cos(th)], 1)


def c3(total):
    import bench
    from fakepta_amd import _capi
    from fakepta import correlated_noises as cn
    from fakepta_amd.batch import BatchSimulator
    ctx = new_context(_capi)
    psrs = bench.build_array(100, 2000, "c2")
    sim = BatchSimulator(psrs, signals=["gw_common"], white=False, ctx=ctx)
    B = 4096
    nb = (total + B - 1) // B
    sums = []

    def step(s):
        n = min(B, total - (s % nb) * B)
        ctx.batch_synth(1234, (s % nb) * B, n, to_host=False)

    dt = timed(ctx, _capi, step, nb, warmup=1)
    sums = ctx.batch_checksums()
    info = ctx.batch_info()
    kt = isolated(ctx, _capi, step, 3)
    del cn
    return dict(config="c3", K=info["K"], realizations=total, batch=B, wall_s=dt, path=ctx.batch_grid_info()["last_path"],
                samples_per_s=info["n_toa"] * total / dt, isolated_kernels_ms_per_batch=kt,
                last_checksum=float(sums[:, 1].sum()),
                note="per-batch device-resident blocks with a full checksum pass (bench.py --config c3 is the "
                     "sharded job with fused checksums)")


def c4_layout(ctx):
    """C4's array on ctx (1000 psr x 10k TOAs, HD100 common signal with the batch path's Cholesky factor); returns
    (P, n_p, N, L)."""
    from fakepta.constants import yr
    from fakepta.spectrum import powerlaw
    P, n_p, N = 1000, 10000, 100
    rng = np.random.default_rng(0)
    T = 10 * yr
    offs = (np.arange(P + 1) * n_p).astype(np.int64)
    toas = (np.linspace(0, T, n_p)[None, :] + rng.uniform(0, 86400, (P, 1))).ravel()
    nu = np.abs(1400.0 + rng.normal(0, 10, P * n_p))
    from fakepta_amd.batch import batch_factor
    class _P:  # noqa: E306
        def __init__(self, p):
            self.pos = p
    from fakepta.correlated_noises import hd
    # the batch path's factor (fakepta_amd.batch.batch_factor, as BatchSimulator): Cholesky of the positive-definite
    # HD ORF, so k_mix_mfma stops each pulsar tile's q loop at its last pulsar (half the FLOPs of the SVD factor)
    L = batch_factor(hd([_P(x) for x in fib(P)]))
    f = np.arange(1, N + 1) / np.ptp(toas)
    amp = np.sqrt(powerlaw(f, -15.0, 13 / 3) * np.diff(np.append(0.0, f)))  # df as fake_pta.py:370
    ctx.batch_set_toas(offs, toas, nu)
    ctx.batch_add_signal(1, f, amp, idx=0.0, L=L)
    return P, n_p, N, L


def c4(steps=5):
    from fakepta_amd import _capi
    ctx = new_context(_capi)
    R = 256
    P, n_p, N, L = c4_layout(ctx)
    dt = timed(ctx, _capi, lambda s: ctx.batch_synth(7, s * R, R, to_host=False), steps, warmup=1)
    kt1 = isolated(ctx, _capi, lambda s: ctx.batch_synth(7, s * R, R, to_host=False), 3)
    flops = 2.0 * 2 * N * P * n_p * R
    gi = ctx.batch_grid_info()
    ctx.close()
    return dict(config="c4", K=2 * N, n_toa=P * n_p, realizations=R, ms_per_step=dt / steps * 1e3,
                samples_per_s=P * n_p * R * steps / dt, isolated_kernels_ms_per_step=kt1,
                interp=_interp_entry(gi, P * n_p, R, kt1["synth"], K=2 * N),
                path=gi["last_path"],
                synth_direct_equiv_tflops=flops / ((kt1["synth"] + kt1["grid"]) / 1e3) / 1e12,
                mix_factor="cholesky" if np.all(np.triu(L, 1) == 0) else "svd",
                mix_ms_isolated=kt1["mix"],
                mix_tflops=(P * (P + 1) if np.all(np.triu(L, 1) == 0) else 2.0 * P * P) * 2 * N * R / (kt1["mix"] / 1e3) / 1e12
                if kt1["mix"] else None)


def c5_layout(ctx):
    """C5's array on ctx (100 psr x 2000 TOAs on two backends: RN30 + DM100 + Sv100, HD + monopole + dipole common
    signals, white + ECORR); returns the BatchSimulator."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd.batch import BatchSimulator
    P = 100
    np.random.seed(7)
    pos = fib(P)
    epochs = np.arange(1, 501) * 7.3 * 86400.0
    psrs = []
    for p in range(P):
        th, ph = np.arccos(pos[p, 2]), np.mod(np.arctan2(pos[p, 1], pos[p, 0]), 2 * np.pi)
        t = np.sort(np.concatenate([epochs, epochs + 3600.0]))
        psr = fp.Pulsar(t, 1e-7, th, ph, backends=["A.1400", "B.800"], custom_model={"RN": 30, "DM": 100, "Sv": 100})
        psr.add_white_noise(add_ecorr=True, randomize=True)
        psr.add_red_noise(log10_A=-14, gamma=3)
        psr.add_dm_noise(log10_A=-14, gamma=3)
        psr.add_chromatic_noise(log10_A=-14, gamma=3)
        psrs.append(psr)
    cn.add_common_correlated_noise(psrs, orf="hd", name="gw", log10_A=-14.5, gamma=13 / 3)
    cn.add_common_correlated_noise(psrs, orf="monopole", name="clk", log10_A=-15.0, gamma=4.0)
    cn.add_common_correlated_noise(psrs, orf="dipole", name="eph", log10_A=-15.0, gamma=4.0)
    return BatchSimulator(psrs, white=True, ecorr=True, ctx=ctx)


def c5(steps=10):
    from fakepta_amd import _capi
    ctx = new_context(_capi)
    sim = c5_layout(ctx)
    R = 1024
    dt = timed(ctx, _capi, lambda s: ctx.batch_synth(9, s * R, R, to_host=False), steps)
    info = ctx.batch_info()
    kt = isolated(ctx, _capi, lambda s: ctx.batch_synth(9, s * R, R, to_host=False), 3)
    gi = ctx.batch_grid_info()
    ctx.close()
    return dict(config="c5", K=info["K"], n_toa=info["n_toa"], realizations=R, ms_per_step=dt / steps * 1e3,
                samples_per_s=info["n_toa"] * R * steps / dt, isolated_kernels_ms_per_step=kt,
                interp=_interp_entry(gi, info["n_toa"], R, kt["synth"], K=info["K"]),
                step_ms_per_gb_written=dt / steps * 1e3 / (8.0 * info["n_toa"] * R / 1e9),
                synth_direct_equiv_tflops=2.0 * info["K"] * info["n_toa"] * R / ((kt["synth"] + kt["grid"]) / 1e3) / 1e12,
                path=gi["last_path"], n_ecorr_blocks=len(sim.blocks))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c1", "c3", "c4", "c5"])
    ap.add_argument("--c3-real", type=int, default=100000)
    ap.add_argument("--opt", action="append", default=[], help="library option NAME=VALUE (e.g. INTERP_WS=4)")
    args = ap.parse_args()
    OPTS.extend(args.opt)
    for c in args.configs:
        res = c3(args.c3_real) if c == "c3" else globals()[c]()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
