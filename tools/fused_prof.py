"""Phase breakdown of k_grid_fused on C2 from its per-wave cycle counters (diagnostic build only):

    make -C fakepta_amd/csrc variant NAME=fprof DEFS=-DFPTA_FUSED_PROF
    FAKEPTA_AMD_LIB=build/diag/lib_fprof.so python tools/fused_prof.py [--overlap 0|1] [--opt NAME=VALUE ...]

Counters per wave (grid_fused.hip Prof): interpolation waves 0 next-chunk loads, 1 MFMA steps, 2 stores, 3 barriers,
4 wide-chunk reloads, 5 chunks; DFT waves 0 tables + draws, 1 MFMA steps, 2 ring sync, 3 grid writes, 4 barriers,
5 groups. Prints the mean over workgroups of each role's waves, in microseconds at the kernel's clock.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--overlap", type=int, default=0)
    ap.add_argument("--blocks", type=int, default=3)
    ap.add_argument("--ghz", type=float, default=2.2, help="clock for the cycle -> time conversion")
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--config", default="c2", choices=["c2", "c4", "c5"])
    args = ap.parse_args()
    from bench import build_array
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator
    fn = getattr(_capi._lib, "fpta_debug_fused_prof", None)
    if fn is None:
        sys.exit("fused_prof.py: the loaded library is not a -DFPTA_FUSED_PROF build")
    ctx = _capi.Context(0)
    if args.config == "c2":
        psrs = build_array(100, 2000, "c2")
        sim = BatchSimulator(psrs, white=False, ctx=ctx)
        R = 1024
        run = lambda b: sim.synth(R, seed=1234, real0=b * R, to_host=False)  # noqa: E731
    elif args.config == "c5":  # C5's layout (tools/bench_configs.py c5): k_grid_fused_w
        from tools.bench_configs import c5_layout
        sim = c5_layout(ctx)
        R = 1024
        run = lambda b: ctx.batch_synth(9, b * R, R, to_host=False)  # noqa: E731
    else:  # C4's layout (tools/bench_configs.py c4): 1000 psr x 10k TOAs, HD100, R = 256
        from tools.bench_configs import c4_layout
        c4_layout(ctx)
        R = 256
        run = lambda b: ctx.batch_synth(7, b * R, R, to_host=False)  # noqa: E731
    ctx.set_option(_capi.OPT_OVERLAP, args.overlap)
    for kv in args.opt:
        k, v = kv.split("=")
        ctx.set_option(getattr(_capi, "OPT_" + k.upper()), int(v))
    for b in range(args.blocks):
        run(b)
    ctx.synchronize()
    print("kernel:", ctx.batch_grid_info()["interp_kernel"])
    n = 4096 * 8 * 8
    buf = (ctypes.c_ulonglong * n)()
    rc = fn(ctx._h, buf, ctypes.c_int64(n))
    if rc:
        sys.exit(f"fpta_debug_fused_prof failed ({rc})")
    v = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8, 8).astype(float)
    used = v.sum(axis=(1, 2)) > 0
    v = v[used]
    cyc_us = 1e-3 / args.ghz
    names = {"interp": ["loads", "mfma", "stores", "barriers", "reloads", "chunks", "stream+info"],
             "dft": ["loads issue", "mfma", "sync/join st", "grid writes", "barr/join wide", "iterations", "draws", "joined chunks"]}
    print(f"workgroups with counters: {len(v)}")
    for role, waves in (("interp", range(0, 4)), ("dft", range(4, 8))):
        r = v[:, list(waves), :]
        print(f"{role} waves (mean over workgroups; per wave):")
        for i, nm in enumerate(names[role]):
            col = r[:, :, i]
            if i >= r.shape[2]:
                continue
            if nm in ("chunks", "iterations", "joined chunks"):
                print(f"   {nm:14s} {col.mean():10.1f}   (per wave: {', '.join(f'{x:.1f}' for x in col.mean(axis=0))})")
            else:
                print(f"   {nm:14s} {col.mean() * cyc_us:10.1f} us   (per wave: "
                      f"{', '.join(f'{x * cyc_us:.1f}' for x in col.mean(axis=0))})")
        tot = r[:, :, :5].sum(axis=2) + r[:, :, 6]
        print(f"   {'total':14s} {tot.mean() * cyc_us:10.1f} us")
    ctx.close()


if __name__ == "__main__":
    main()
