"""Diagnostic timing of the gridded interpolation kernel on C2 (not part of the product or the bench).

    FAKEPTA_AMD_LIB=<lib.so> python tools/interp_diag.py [--grid-mfma M]

Prints the average k_grid_interp_mfma and k_grid_dft launch times (HIP events on the context stream) over 10
batches of 1024 realizations, and the plan figures. FAKEPTA_AMD_LIB selects a diagnostic build of the library
(never the bench)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid-mfma", type=int, default=-1)
    ap.add_argument("--label", default="")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--ws", type=int, default=-1, help="FPTA_OPT_INTERP_WS (-1: library default)")
    ap.add_argument("--overlap", type=int, default=0, help="FPTA_OPT_OVERLAP (1: pipelined blocks, co-running DFT)")
    args = ap.parse_args()
    import bench
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator
    ctx = _capi.Context(0)
    psrs = bench.build_array(100, 2000, "c2")
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    ctx.set_option(_capi.OPT_SYNTH_PATH, 4)
    ctx.set_option(_capi.OPT_OVERLAP, args.overlap)  # 0: the kernels alone (no co-running draws of the next batch)
    if args.grid_mfma >= 0:
        ctx.set_option(_capi.OPT_GRID_MFMA, args.grid_mfma)
    if args.ws >= 0:
        ctx.set_option(_capi.OPT_INTERP_WS, args.ws)
    if args.width:
        ctx.set_option(_capi.OPT_GRID_WIDTH, args.width)
    for i in range(3):
        sim.synth(1024, seed=1, real0=i * 1024, to_host=False)
    ctx.synchronize()
    ctx.set_option(_capi.OPT_PROFILE, 1)
    ctx.reset_stats()
    import time
    t0 = time.perf_counter()
    for i in range(10):
        sim.synth(1024, seed=1, real0=(3 + i) * 1024, to_host=False)
    ctx.synchronize()
    step_ms = (time.perf_counter() - t0) * 100
    n, ms = ctx.kernel_stats(_capi.K_SYNTH)
    nd, msd = ctx.kernel_stats(_capi.K_GRID)
    print(json.dumps({"label": args.label, "lib": os.path.basename(_capi.LIB_PATH), "interp_ms": ms / n,
                      "dft_ms": msd / max(nd, 1), "step_ms": step_ms, "grid": ctx.batch_grid_info()}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
