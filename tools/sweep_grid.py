"""Interleaved A/B of the gridded-path kernels on the C2 workload (one process, HIP-event timing).

    python tools/sweep_grid.py [--rounds 5] [--reps 5] [--real 1024] [--masks 0,1]
                               [--params 13:200,11:150,...]

mask = FPTA_OPT_GRID_MFMA: 1 runs k_grid_dft on MFMA, 0 on VALU (the interpolation always runs on MFMA).
Prints per mask the median k_grid_dft and interpolation times, and the max relative deviation of
the output from the exact seeded VALU path (path 3) on the same device coefficients.
--params sweeps (kernel width w, oversampling sigma x 100) pairs instead, at the first mask.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--real", type=int, default=1024)
    ap.add_argument("--masks", default="0,1")
    ap.add_argument("--params", default="", help="w:sigma100 pairs, e.g. 13:200,11:150")
    args = ap.parse_args()
    import bench
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator

    ctx = _capi.Context(0)
    psrs = bench.build_c2(100, 2000)
    BatchSimulator(psrs, white=False, ctx=ctx)
    R = args.real
    masks = [int(m) for m in args.masks.split(",")]
    if args.params:  # (width, sigma) configurations at the first mask
        cfgs = [(masks[0],) + tuple(int(v) for v in p.split(":")) for p in args.params.split(",")]
    else:
        cfgs = [(m, 15, 150) for m in masks]

    def apply(cfg):
        ctx.set_option(_capi.OPT_GRID_MFMA, cfg[0])
        ctx.set_option(_capi.OPT_GRID_WIDTH, cfg[1])
        ctx.set_option(_capi.OPT_GRID_SIGMA, cfg[2])

    ctx.set_option(_capi.OPT_SYNTH_PATH, 3)
    exact = ctx.batch_synth(1234, 0, R, to_host=True)
    ctx.set_option(_capi.OPT_SYNTH_PATH, 4)
    dev = {}
    for cfg in cfgs:
        apply(cfg)
        out = ctx.batch_synth(1234, 0, R, to_host=True)
        dev[cfg] = float(np.max(np.abs(out - exact)) / np.max(np.abs(exact)))
    times = {cfg: ([], []) for cfg in cfgs}
    ctx.set_option(_capi.OPT_PROFILE, 1)
    for rnd in range(args.rounds):
        for cfg in cfgs:
            apply(cfg)
            ctx.batch_synth(1234, 0, R, to_host=False)  # rebuild the layout outside the timed reps
            ctx.reset_stats()
            for i in range(args.reps):
                ctx.batch_synth(1234, (rnd * args.reps + i) * R, R, to_host=False)
            n, ms = ctx.kernel_stats(_capi.K_GRID)
            times[cfg][0].append(ms / max(n, 1))
            n, ms = ctx.kernel_stats(_capi.K_SYNTH)
            times[cfg][1].append(ms / max(n, 1))
    for cfg in cfgs:
        d, s = np.array(times[cfg][0]), np.array(times[cfg][1])
        print(json.dumps(dict(mask=cfg[0], width=cfg[1], sigma100=cfg[2], dft_ms_median=float(np.median(d)),
                              interp_ms_median=float(np.median(s)), sum_ms=float(np.median(d) + np.median(s)),
                              max_rel_dev_vs_exact=dev[cfg])), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
