"""Interleaved A/B of the synthesis kernels on the C2 workload (one process, HIP-event timing).

    python tools/sweep_synth.py [--rounds 5] [--reps 5] [--real 1024]

Prints per-variant median/min synth-kernel time and TFLOP/s (algorithmic 2*K flops per sample),
plus the max relative deviation of each variant's output from the MFMA path's.
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
    ap.add_argument("--variants", default="mfma,valu0,valu1,valu2,valu3,valu4,valu5")
    ap.add_argument("--anchors", default="0")
    args = ap.parse_args()
    import bench
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator

    ctx = _capi.Context(0)
    psrs = bench.build_c2(100, 2000)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    info = ctx.batch_info()
    R = args.real
    flops = 2.0 * info["K"] * info["n_toa"] * R
    configs = []
    for v in args.variants.split(","):
        for a in args.anchors.split(","):
            configs.append((v, int(a)))

    def setup(v, anchor):
        ctx.set_option(_capi.OPT_ANCHOR, anchor)
        if v == "mfma":
            ctx.set_option(_capi.OPT_SYNTH_PATH, 2)
        else:
            ctx.set_option(_capi.OPT_SYNTH_PATH, 3)
            ctx.set_option(_capi.OPT_VALU_VARIANT, int(v[4:]))

    ref = None
    dev = {}
    for v, a in configs:
        setup(v, a)
        out = ctx.batch_synth(1234, 0, R, to_host=True)
        if ref is None:
            ref = out
        dev[(v, a)] = float(np.max(np.abs(out - ref)) / np.max(np.abs(ref)))
    times = {c: [] for c in configs}
    ctx.set_option(_capi.OPT_PROFILE, 1)
    for rnd in range(args.rounds):
        for c in configs:
            setup(*c)
            ctx.reset_stats()
            for i in range(args.reps):
                ctx.batch_synth(1234, (rnd * args.reps + i) * R, R, to_host=False)
            n, ms = ctx.kernel_stats(_capi.K_SYNTH)
            times[c].append(ms / n)
    res = []
    for c in configs:
        t = np.array(times[c])
        res.append(dict(variant=c[0], anchor=c[1], median_ms=float(np.median(t)), min_ms=float(t.min()),
                        tflops_median=flops / np.median(t) / 1e9, max_rel_dev_vs_first=dev[c]))
        print(json.dumps(res[-1]), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
