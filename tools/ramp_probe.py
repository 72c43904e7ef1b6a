"""Per-step times of the C2 step from a cold start, and after ~0.3 s of other GPU work (the exact path on the same
batch): is the warmup ramp of k_grid_fused a property of the GPU's state or of the data path?
    python tools/ramp_probe.py [--steps 60]
Each step is synchronized (its wall time includes one host round trip)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    args = ap.parse_args()
    from bench import build_array
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator
    ctx = _capi.Context(0)
    sim = BatchSimulator(build_array(100, 2000, "c2"), white=False, ctx=ctx)
    R = 1024

    def run(tag, n, real0):
        ts = []
        for s in range(n):
            t0 = time.perf_counter()
            sim.synth(R, seed=1234, real0=real0 + s * R, to_host=False)
            ctx.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        print(tag, " ".join(f"{t:.3f}" for t in ts), flush=True)

    sim.synth(R, seed=1234, real0=0, to_host=False)  # plan, buffers
    ctx.synchronize()
    time.sleep(1.0)
    run("cold", args.steps, R)
    time.sleep(1.0)
    ctx.set_option(_capi.OPT_SYNTH_PATH, 3)  # ~0.3 s of the exact path first
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        sim.synth(R, seed=1234, real0=0, to_host=False)
        ctx.synchronize()
    ctx.set_option(_capi.OPT_SYNTH_PATH, 0)
    run("after_exact", args.steps, 10 ** 6)
    ctx.close()


if __name__ == "__main__":
    main()
