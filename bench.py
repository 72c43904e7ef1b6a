"""Benchmark: BASELINE.json metric on configs[1] (C2), one MI355X per rank.

Workload: 100 pulsars (Fibonacci sky) x 2000 TOAs, per-pulsar power-law
red noise (30 modes) + DM noise (100 modes, nu^-2) + Hellings-Downs-correlated common GWB
(30 modes, log10_A = -15, gamma = 13/3); K = 320 basis columns. One step = 1024 new
realizations per GPU drawn on device (Philox -> ORF mix -> fused MFMA synthesis), written
to a resident [1024 x 200000] fp64 residual block in HBM. Inputs are resident before the
timed region; nothing is copied back inside it.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)

Realizations shard across ranks with no data-path collective (weak scaling: rank g of G owns
realizations (step * G + g) * R ...); RCCL is used for the barrier, the max-over-ranks time and
a gather of per-realization checksums to rank 0.
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "residual samples/sec (TOA×realization) for 100-psr HD GWB; % FP64 peak"
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix (= vector) peak, AMD datasheet (MI355X_MICROARCH.md lists none)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SYNTH_KERNELS = {3: ("k_synth_valu_seeded<2,16>", "fp64-valu"), 2: ("k_synth_mfma<4,2>", "fp64-mfma"),
                 1: ("k_synth_direct", "fp64-valu")}
GRID_INTERP = {True: ("k_grid_interp_mfma<8>", "fp64-mfma"), False: ("k_grid_interp<16>", "fp64-valu")}
GRID_DFT = {True: "k_grid_dft_mfma<2,2>", False: "k_grid_dft<8>"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--real", type=int, default=1024, help="realizations per GPU per step")
    ap.add_argument("--npsr", type=int, default=100)
    ap.add_argument("--ntoa", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-sample", type=int, default=8, help="realizations timed for the CPU baseline (0: skip)")
    ap.add_argument("--path", type=int, default=0, help="synthesis path: 0 auto, 1 direct, 2 MFMA, 3 VALU, 4 gridded")
    ap.add_argument("--anchor", type=int, default=0, help="recurrence re-anchor interval (0: library default)")
    ap.add_argument("--grid-mfma", type=int, default=-1,
                    help="gridded path kernels on MFMA: bit 0 DFT, bit 1 interpolation (-1: library default)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL on ROCm) or gloo (CPU rehearsal)")
    ap.add_argument("--traffic", default="",
                    help="PMC-derived HBM bytes per synth launch (written by profiles/collect_pmc.py); "
                         "default: the profiles/*traffic.json record matching the kernel and shape")
    return ap.parse_args()


# --------------------------------------------------------------------------- distributed helpers
def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def shard_range(n_real, rank, world, step):
    """Global realization indices of `rank` at `step` (weak scaling; invariant realization ids)."""
    start = (step * world + rank) * n_real
    return start, n_real


class Comm:
    """Barrier / max / gather over torch.distributed (RCCL on GPUs, gloo on CPU tests)."""

    def __init__(self, world, rank, local, backend=None, device=None):
        self.world, self.rank = world, rank
        self.dist = None
        if world > 1:
            import torch
            import torch.distributed as dist
            if backend is None:
                backend = "nccl"
            if backend == "nccl":
                torch.cuda.set_device(local)
                self.device = torch.device("cuda", local)
            else:
                self.device = torch.device("cpu")
            if not dist.is_initialized():
                dist.init_process_group(backend=backend)
            self.dist = dist
            self.torch = torch

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        if not self.dist:
            return x
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, arr):
        """All ranks' arrays (same shape) stacked on every rank, in rank order."""
        if not self.dist:
            return arr[None]
        t = self.torch.from_numpy(np.ascontiguousarray(arr)).to(self.device)
        bufs = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(bufs, t)
        return np.stack([b.cpu().numpy() for b in bufs])

    def close(self):
        if self.dist and self.dist.is_initialized():
            self.dist.destroy_process_group()


# --------------------------------------------------------------------------- workload
def build_c2(n_psr, n_toa):
    """C2 array through the drop-in API (make_fake_array + add_common_correlated_noise, seed 0)."""
    from fakepta_amd import correlated_noises as cn
    from fakepta_amd import fake_pta as fp
    np.random.seed(0)
    psrs = fp.make_fake_array(npsrs=n_psr, Tobs=10, ntoas=n_toa, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": 100, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3, components=30)
    return psrs


def cpu_baseline(sim, psrs, n_sample, seed):
    """Oracle (numpy restatement, loop-faithful to fake_pta.py:385-387 / correlated_noises.py:153-160)
    timed on this host, 1 thread, for `n_sample` realizations of the same workload."""
    from oracle import fakepta_oracle as O
    P = len(psrs)
    segs = sim.segments
    t0 = time.perf_counter()
    for r in range(n_sample):
        rng = np.random.default_rng(seed + r)
        res = [np.zeros(len(p.toas)) for p in psrs]
        for s in segs:
            if s["kind"] == 0:
                for p in range(P):
                    nm = s["f"].shape[1]
                    amp = s["amp"][p]
                    psd = amp ** 2 / O.delta_f(s["f"][p])
                    coeffs = O.gp_coeffs_from_z(psd, rng.standard_normal(2 * nm))
                    O.gp_synth_loop(psrs[p].toas, psrs[p].freqs, s["f"][p], coeffs, s["idx"], residuals=res[p])
            else:
                nm = len(s["f"])
                psd = s["amp"] ** 2 / O.delta_f(s["f"])
                z = rng.standard_normal((nm, 2, P))
                out, _ = O.common_synth_loop([p.toas for p in psrs], [p.freqs for p in psrs], s["f"], psd, z,
                                             s["L"], s["idx"])
                for p in range(P):
                    res[p] += out[p]
    dt = time.perf_counter() - t0
    n_samples = sim.n_toa * n_sample
    return dict(value=n_samples / dt, unit="samples/s", cores=1, kind="port",
                sample=f"{n_sample} realizations of the C2 array (100 psr x 2000 TOAs, RN30+DM100+HD30), "
                       f"oracle loop-faithful restatement, numpy {np.__version__}, 1 thread, "
                       f"{dt:.2f} s on {os.cpu_count()}-CPU host")


def main():
    args = parse()
    world, rank, local = dist_env()
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator

    # one process per GPU; local ranks beyond the visible devices wrap (rehearsal of several ranks on
    # one card with --dist-backend gloo; the driver's N-GPU runs have one rank per device)
    ndev = max(1, _capi.device_count())
    device = local % ndev
    os.environ["FAKEPTA_AMD_DEVICE"] = str(device)  # the drop-in calls of build_c2 use the same card
    comm = Comm(world, rank, device, backend=args.dist_backend)
    ctx = _capi.Context(device)
    psrs = build_c2(args.npsr, args.ntoa)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    info = ctx.batch_info()
    if args.path:
        ctx.set_option(_capi.OPT_SYNTH_PATH, args.path)
    if args.anchor:
        ctx.set_option(_capi.OPT_ANCHOR, args.anchor)
    if args.grid_mfma >= 0:
        ctx.set_option(_capi.OPT_GRID_MFMA, args.grid_mfma)
    R = args.real

    for s in range(args.warmup):
        real0, n = shard_range(R, rank, world, s)
        ctx.batch_synth(args.seed, real0, n, to_host=False)
    ctx.synchronize()
    ctx.set_option(_capi.OPT_PROFILE, 1)
    ctx.reset_stats()

    comm.barrier()
    ctx.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        real0, n = shard_range(R, rank, world, args.warmup + s)
        ctx.batch_synth(args.seed, real0, n, to_host=False)
    ctx.synchronize()
    comm.barrier()
    dt_local = time.perf_counter() - t0
    dt = comm.max(dt_local)

    ctx.set_option(_capi.OPT_PROFILE, 0)
    kstats = {name: ctx.kernel_stats(k) for name, k in
              (("gen", _capi.K_GEN), ("mix", _capi.K_MIX), ("grid", _capi.K_GRID), ("synth", _capi.K_SYNTH),
               ("white", _capi.K_WHITE))}
    sums = ctx.batch_checksums()  # last step's realizations
    all_sums = comm.gather(sums)
    n_samples_total = info["n_toa"] * R * args.steps * world
    value = n_samples_total / dt

    synth_n, synth_ms = kstats["synth"]
    synth_avg_s = synth_ms / max(synth_n, 1) / 1e3
    flops = 2.0 * info["K"] * info["n_toa"] * R
    gi = ctx.batch_grid_info()
    path = gi["last_path"]
    if path == 4:
        kernel, pipe = GRID_INTERP[bool(gi["grid_mfma"] & 2)]
    else:
        kernel, pipe = SYNTH_KERNELS[path]
    traffic = None
    candidates = ([args.traffic] if args.traffic else
                  sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic.json"))))
    for cand in candidates:
        try:
            with open(cand) as fh:
                tr = json.load(fh)
        except (OSError, ValueError):
            continue
        # a PMC record only counts for the same kernel on the same shape (same launch)
        if (tr.get("K") == info["K"] and tr.get("n_real") == R and tr.get("n_toa") == info["n_toa"]
                and kernel.startswith(tr.get("kernel", "?"))):
            traffic = tr.get("hbm_bytes_per_launch")
            break
    out_bytes = 8.0 * info["n_toa"] * R
    if path == 4:
        # gridded path: the dominant kernel is the interpolation, an HBM-bound stream:
        # algorithmic bytes = residual block written once + grid values read once + interpolation weights
        R_pad = -(-R // 128) * 128
        alg_bytes = out_bytes + 8.0 * gi["grid_vals"] * R_pad + gi["weight_bytes"]
        achieved = alg_bytes / synth_avg_s / 1e9
        grid_n, grid_ms = kstats["grid"]
        grid_avg_s = grid_ms / max(grid_n, 1) / 1e3
        dft_flops = 2.0 * gi["fma_dft"] * R_pad
        roofline = {"bound": "hbm", "pipe": pipe, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kernel,
                    "bytes_per_launch": alg_bytes, "avg_launch_ms": synth_avg_s * 1e3,
                    "write_GBps": out_bytes / synth_avg_s / 1e9,
                    "interp_fp64_TFLOPs": 2.0 * gi["fma_interp"] * R_pad / synth_avg_s / 1e12,
                    "dft": {"kernel": GRID_DFT[bool(gi["grid_mfma"] & 1)], "avg_launch_ms": grid_avg_s * 1e3,
                            "flops_per_launch": dft_flops, "TFLOPs": dft_flops / max(grid_avg_s, 1e-12) / 1e12,
                            "frac_fp64_peak": dft_flops / max(grid_avg_s, 1e-12) / 1e12 / FP64_PEAK_TFLOPS},
                    "direct_equivalent_TFLOPs": flops / (synth_avg_s + grid_avg_s) / 1e12}
    else:
        # exact paths: compute (FP64) bound, 2K FLOP per 8-byte sample = 80 FLOP/B at K = 320. The peak is
        # the MI355X FP64 datasheet figure, equal for the vector and matrix pipes (DESIGN.md §5 Calibration)
        achieved = flops / synth_avg_s / 1e12
        roofline = {"bound": "mfma", "pipe": pipe, "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "kernel": kernel,
                    "flops_per_launch": flops, "avg_launch_ms": synth_avg_s * 1e3,
                    "write_GBps": out_bytes / synth_avg_s / 1e9}

    if rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": "C2 (BASELINE configs[1]): %d psr x %d TOAs, RN30 + DM100(nu^-2) + HD GWB30, "
                                   "%d realizations/GPU/step, Philox seed %d" % (args.npsr, args.ntoa, R, args.seed),
                       "n_psr": args.npsr, "n_toa_total": info["n_toa"], "K": info["K"], "realizations_per_gpu": R,
                       "parallelism": "realization-sharded x%d" % world},
            "synth_path": {1: "direct", 2: "mfma", 3: "valu-seeded", 4: "gridded"}.get(path, str(path)),
            "roofline": roofline,
            "kernels_ms_per_step": {k: (v[1] / max(v[0], 1)) * (v[0] / max(args.steps, 1)) for k, v in kstats.items()},
            "checksum": float(np.sum(all_sums[..., 1])),
        }
        if world == 1 and args.cpu_sample > 0:
            line["cpu_baseline"] = cpu_baseline(sim, psrs, args.cpu_sample, args.seed)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    ctx.close()
    comm.close()


if __name__ == "__main__":
    main()
