"""Is the C2 warmup ramp the shader clock? Per step of a cold start: the fused launch's duration (its
dispatch-bound HIP events) and its interpolation waves' shader-clock cycles (FPTA_FUSED_PROF counters, s_memtime), whose
ratio is the clock the launch ran at. Diagnostic build only:

    make -C fakepta_amd/csrc variant NAME=fprof DEFS=-DFPTA_FUSED_PROF
    FAKEPTA_AMD_LIB=build/diag/lib_fprof.so python tools/ramp_clock_probe.py [--steps 80]
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
    ap.add_argument("--steps", type=int, default=80)
    args = ap.parse_args()
    from bench import build_array
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator
    fn = getattr(_capi._lib, "fpta_debug_fused_prof", None)
    if fn is None:
        sys.exit("ramp_clock_probe.py: the loaded library is not a -DFPTA_FUSED_PROF build")
    ctx = _capi.Context(0)
    sim = BatchSimulator(build_array(100, 2000, "c2"), white=False, ctx=ctx)
    R = 1024
    ctx.set_option(_capi.OPT_PROFILE, 1)
    n = 4096 * 8 * 8
    buf = (ctypes.c_ulonglong * n)()
    print("step  launch_ms  interp_wave_Mcycles  clock_GHz")
    prev_n, prev_ms = 0, 0.0
    for s in range(args.steps):
        sim.synth(R, seed=1234, real0=s * R, to_host=False)
        ctx.synchronize()
        cnt, tot = ctx.kernel_stats(_capi.K_SYNTH)
        ms = (tot - prev_ms) / max(1, cnt - prev_n)
        prev_n, prev_ms = cnt, tot
        if fn(ctx._h, buf, ctypes.c_int64(n)):
            sys.exit("fpta_debug_fused_prof failed")
        v = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8, 8).astype(float)
        used = v.sum(axis=(1, 2)) > 0
        cyc = v[used][:, 0:4, :5].sum(axis=2).mean()  # interpolation waves: every timed phase
        print(f"{s:4d}  {ms:9.4f}  {cyc / 1e6:19.4f}  {cyc / (ms * 1e6):9.3f}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
