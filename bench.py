"""Benchmark: the BASELINE.json metric, one MI355X per rank.

Default workload = C2 (BASELINE configs[1]): 100 pulsars (Fibonacci sky) x 2000
TOAs, per-pulsar power-law red noise (30 modes) + DM noise (100 modes, nu^-2) + Hellings-Downs-
correlated common GWB (30 modes, log10_A = -15, gamma = 13/3); K = 320 basis columns. One step =
1024 new realizations per GPU drawn on device (Philox -> ORF mix -> synthesis), written to a
resident [1024 x 200000] fp64 residual block in HBM. Inputs are resident before the timed region;
nothing is copied back inside it. Weak scaling: rank g of G owns realizations (step G + g) R ...
The step's launches: k_gen_mix (the GWB draws + HD mix) and k_grid_fused (per-pulsar draws, the grid DFTs into LDS and
the interpolation, one persistent kernel); the roofline block names the dominant kernel as the library reports it.

--config c3 (BASELINE configs[2]): the same 100-psr array with the HD GWB only (K = 60), a job of
100,000 realizations sharded over the ranks (fakepta_amd.batch.simulate_sharded: rank g owns
[g R/G, (g+1) R/G)), streamed in batches of 7168 per GPU, per-realization checksums gathered to
rank 0. Strong scaling (the job is fixed); one step = the whole job.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3]
    (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N; run without a launcher,
    --gpus N > 1 starts that launcher as a child process before anything touches a GPU)

One process per GPU. RCCL over xGMI (the library's own communicator, fpta_comm_*, on the kernels' HIP runtime;
fakepta_amd.batch.RcclComm) carries only the barrier, the max-over-ranks time and the checksum gather; the data
path has no collective. The rank processes never import torch (one HIP runtime per process).
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


def grid_interp_kernel(ws, part, r_pad):
    """Name of the interpolation kernel FPTA_OPT_INTERP_WS = ws launches for plain (C2) or fused-checksum (C3) blocks
    of R_pad realizations (the default takes the 256-realization tiles of k_grid_interp_ws2 when they waste fewer
    realization slots than the 512 of k_grid_interp_ws, as capi.hip does)."""
    p = "true" if part else "false"
    reg = f"k_grid_interp_mfma<false, {p}, 8>"
    if ws == 1 and not part and -(-r_pad // 256) * 256 - r_pad < -(-r_pad // 512) * 512 - r_pad:
        ws = 3
    return {0: reg, 1: reg if part else "k_grid_interp_ws<false>", 2: f"k_grid_interp_ws<{p}>",
            3: reg if part else "k_grid_interp_ws2<false>", 4: f"k_grid_interp_st<false, {p}>"}[ws]


# layout tag of the gridded plan a PMC traffic record must carry to describe the shipped interpolation kernel
# (32-TOA chunks, every grid signal's band back to back, coalesced signals); older tags describe earlier plans
GRID_LAYOUT = "band32c"
GRID_DFT = {True: "k_grid_dft_mfma<2,2>", False: "k_grid_dft<8>"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=("c2", "c3"))
    ap.add_argument("--real", type=int, default=1024, help="c2: realizations per GPU per step")
    ap.add_argument("--c3-real", type=int, default=100000, help="c3: realizations of the whole job")
    # 7168 = 112 blocks of 64 realizations: 100 pulsars x 112 = 11200 k_grid_interp_psr workgroups, 21.9 rounds of
    # the 512 the chip holds (4096: 12.5 rounds, half of the last one idle); 37.8-38.1 vs 39.5-39.6 ms per job on
    # one box (profiles/round4/R5v_c3_batch_sizes.txt). The checksums do not depend on the batch size.
    ap.add_argument("--c3-batch", type=int, default=7168, help="c3: realizations per batch per GPU")
    ap.add_argument("--npsr", type=int, default=100)
    ap.add_argument("--ntoa", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-sample", type=int, default=4,
                    help="re-drawn realizations timed for the reference-faithful CPU baseline (0: skip both CPU legs)")
    ap.add_argument("--path", type=int, default=0, help="synthesis path: 0 auto, 1 direct, 2 MFMA, 3 VALU, 4 gridded")
    ap.add_argument("--grid-mfma", type=int, default=-1,
                    help="gridded path kernels on MFMA: bit 0 DFT, bit 1 interpolation (-1: library default)")
    ap.add_argument("--interp-ws", type=int, default=-1,
                    help="gridded interpolation kernel: 1 warp-specialised, 0 register-pipelined (-1: library default)")
    ap.add_argument("--no-kernel-events", action="store_true",
                    help="diagnostic: no per-kernel HIP events in the timed region (the roofline's launch time is then "
                         "unmeasured; for the events' own cost)")
    ap.add_argument("--event-every", type=int, default=4,
                    help="c2: per-kernel HIP events on every N-th timed step (steps 0, N, 2N, ...): the roofline's "
                         "average launch time from those launches (events put ~10 us of command-processor work "
                         "between two launches, profiles/round6/r6_kernel_events_cost.txt); 1 = every step")
    ap.add_argument("--overlap", type=int, default=-1,
                    help="FPTA_OPT_OVERLAP: 1 pipelined blocks (side stream), 0 one stream (-1: library default)")
    ap.add_argument("--opt", action="append", default=[],
                    help="library option NAME=VALUE (e.g. DFT_GEN=0, GEN_MIX=0, INTERP_WS=2) for A/B runs; repeatable")
    ap.add_argument("--exact-launches", type=int, default=5,
                    help="launches of the exact fused kernel (path 3) timed after the run for roofline_exact")
    ap.add_argument("--dist-backend", default="rccl", choices=("rccl", "gloo"),
                    help="rccl: the library's RCCL communicator (one rank per GPU); gloo: torch.distributed on the "
                         "CPU (rehearsal of several ranks on one card)")
    ap.add_argument("--sub-configs", type=int, default=1,
                    help="c2 at N = 1: after the timed region, compact C3 / C5 / C4-per-GPU records (keys c3, c5, "
                         "c4_per_gpu of the line; tools/bench_configs.sub_records); 0 skips them")
    ap.add_argument("--traffic", default="",
                    help="PMC-derived HBM bytes per launch (profiles/*traffic.json, tools/collect_traffic.py); "
                         "default: the record matching the kernel and shape")
    return ap.parse_args()


def refuse_debug_environment():
    """A measurement must run the release library with no debug switch: refuse FPTA_* variables (the
    release build reads none; a stale one signals a debugging session) and the debug build."""
    bad = sorted(k for k in os.environ if k.startswith("FPTA_"))
    if bad:
        sys.exit(f"bench.py: refusing to measure with debug variables set: {', '.join(bad)}")
    from fakepta_amd import _capi
    if _capi.build_flags() & _capi.BUILD_DEBUG:
        sys.exit(f"bench.py: refusing to measure the debug build ({_capi.LIB_PATH})")


# --------------------------------------------------------------------------- workloads
def build_array(n_psr, n_toa, config):
    """C2 / C3 array through the drop-in API (make_fake_array + add_common_correlated_noise, seed 0)."""
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    np.random.seed(0)
    model = {"RN": 30, "DM": 100, "Sv": None} if config == "c2" else {"RN": None, "DM": None, "Sv": None}
    psrs = fp.make_fake_array(npsrs=n_psr, Tobs=10, ntoas=n_toa, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model=model)
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3, components=30)
    return psrs


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def baseline_segments(sim):
    """The bench layout as the reference's injectors see it: per-pulsar (f, psd) and the common signal's (f, psd, ORF)
    (psd = amp^2 / df; the ORF = L L^T of the batch factor)."""
    from oracle import fakepta_oracle as O
    segs = []
    for s in sim.segments:
        if s["kind"] == 0:
            df = np.diff(np.concatenate([np.zeros((s["f"].shape[0], 1)), s["f"]], 1), axis=1)
            segs.append(dict(kind=0, f=s["f"], psd=s["amp"] ** 2 / df, idx=s["idx"]))
        else:
            segs.append(dict(kind=1, f=s["f"], psd=s["amp"] ** 2 / O.delta_f(s["f"]), idx=s["idx"],
                             orf=s["L"] @ s["L"].T))
    return segs


def cpu_baseline_loop(toas_list, freqs_list, segs, n_sample, seed):
    """n_sample re-drawn realizations with the reference's own operations at its cost, 1 thread
    (oracle.redraw_loop: per mode elementwise passes, the stored signal's reconstruct subtracted before each re-draw
    as fake_pta.py:266-267 / correlated_noises.py:133-134 do, an SVD of the ORF per multivariate_normal call). The
    first realization (no stored signal yet) is not timed. Returns seconds per realization."""
    from oracle import fakepta_oracle as O
    rs = np.random.RandomState(seed)
    res = [np.zeros(len(t)) for t in toas_list]
    stored = {}
    with _one_thread() as used:
        O.redraw_loop(toas_list, freqs_list, segs, res, stored, rs)
        t0 = time.perf_counter()
        for _ in range(n_sample):
            O.redraw_loop(toas_list, freqs_list, segs, res, stored, rs)
        dt = (time.perf_counter() - t0) / n_sample
    return dt, used


class _one_thread:
    """numpy's BLAS / LAPACK pools limited to one thread (threadpoolctl) for the reference-faithful loop (the SVD
    inside each multivariate_normal would otherwise take every OMP thread); yields the BLAS threads in force."""

    def __enter__(self):
        self._lim = None
        try:
            from threadpoolctl import threadpool_limits
            self._lim = threadpool_limits(limits=1)
        except Exception:
            pass
        return blas_threads()

    def __exit__(self, *exc):
        if self._lim is not None:
            self._lim.restore_original_limits()
        return False


def blas_threads():
    """Threads numpy's BLAS actually runs with (threadpoolctl), or None."""
    try:
        from threadpoolctl import threadpool_info
        n = [i.get("num_threads") for i in threadpool_info() if i.get("user_api") == "blas"]
        return max(n) if n else None
    except Exception:
        return None


def cpu_baseline_vectorised(sim, psrs, n_real, seed):
    """the vectorised F.A restatement on the threads numpy's BLAS runs with: per pulsar the
    basis F [n_p x K_p] (built once per batch, as a CPU user would), the draws, the ORF mix x = L z and one GEMM
    F @ A [K_p x n_real]."""
    from oracle import fakepta_oracle as O
    P = len(psrs)
    rng = np.random.default_rng(seed)
    t0 = time.perf_counter()
    zc = {}
    for i, s in enumerate(sim.segments):
        if s["kind"] == 1:
            nm = len(s["f"])
            z = rng.standard_normal((P, 2 * nm * n_real))
            zc[i] = (s["L"] @ z).reshape(P, 2 * nm, n_real)
    for p in range(P):
        out = np.zeros((len(psrs[p].toas), n_real))
        for i, s in enumerate(sim.segments):
            f = s["f"][p] if s["kind"] == 0 else s["f"]
            amp = s["amp"][p] if s["kind"] == 0 else s["amp"]
            F = O.fourier_basis(psrs[p].toas, psrs[p].freqs, f, s["idx"])
            if s["kind"] == 0:
                A = rng.standard_normal((2 * len(f), n_real))
            else:
                A = zc[i][p]
            A *= np.repeat(amp, 2)[:, None]
            out += F @ A
    return time.perf_counter() - t0


def cpu_baseline(sim, psrs, n_sample, seed):
    n_toa = sim.n_toa
    segs = baseline_segments(sim)
    dt_loop, loop_threads = cpu_baseline_loop([p.toas for p in psrs], [p.freqs for p in psrs], segs, n_sample, seed)
    threads = os.environ.get("OMP_NUM_THREADS", "")
    n_vec = 64
    dt_vec = cpu_baseline_vectorised(sim, psrs, n_vec, seed)
    while dt_vec < 2.0 and n_vec < 4096:  # grow the sample to a few seconds of CPU work
        n_vec *= 4
        dt_vec = cpu_baseline_vectorised(sim, psrs, n_vec, seed)
    used = blas_threads()
    vec = dict(value=n_toa * n_vec / dt_vec, unit="samples/s", cores=used, kind="port",
               sample=f"{n_vec} realizations, vectorised F.A (numpy {np.__version__} BLAS GEMM per pulsar), "
                      f"{dt_vec:.2f} s on {used} BLAS thread(s) (OMP_NUM_THREADS={threads or 'unset'}; the GPU "
                      f"box's CPU share is 16 of its {os.cpu_count()} host CPUs)")
    return dict(value=n_toa / dt_loop, unit="samples/s", cores=loop_threads or 1, kind="port",
                blas_threads_in_loop=loop_threads,
                sample=f"{n_sample} re-drawn realizations of the bench array with the reference's operations "
                       f"(oracle.redraw_loop: fake_pta.py:266-267 + 370-387, correlated_noises.py:133-134 + "
                       f"146-160, SVD per multivariate_normal), BLAS limited to {loop_threads} thread(s) "
                       f"(threadpoolctl), {dt_loop:.2f} s per realization; "
                       f"same-host ratio to the reference itself: profiles/r03_cpu_crosscheck.json",
                cpu_model=cpu_model(), nproc=os.cpu_count(), omp_num_threads=threads or None,
                vectorised_blas_threads=vec)


def pmc_traffic(kernel, info, R, path_arg, layout=None):
    """HBM bytes per launch from the matching profiles/*traffic.json PMC record (same kernel, shape and, for the
    gridded path, plan layout)."""
    # newest round first: profiles/roundN/ (N descending), then the earlier rounds' profiles/rNN<letter>_* (a later tag
    # sorts after an earlier one)
    rounds = sorted(glob.glob(os.path.join(ROOT, "profiles", "round*", "*traffic.json")), reverse=True)
    candidates = ([path_arg] if path_arg else
                  rounds + sorted(glob.glob(os.path.join(ROOT, "profiles", "*traffic.json")), reverse=True))
    for cand in candidates:
        try:
            with open(cand) as fh:
                tr = json.load(fh)
        except (OSError, ValueError):
            continue
        if (tr.get("K") == info["K"] and tr.get("n_real") == R and tr.get("n_toa") == info["n_toa"]
                and kernel.startswith(tr.get("kernel", "?")) and tr.get("layout") == layout):
            return tr.get("hbm_bytes_per_launch"), os.path.relpath(cand, ROOT)
    return None, None


def next_mix_mfmas(P, nm, R_pad, lower=True, n_q=None):
    """fp64 MFMAs k_grid_fused runs for the next block's common-signal mix (FPTA_OPT_FUSED_NEXT_MIX,
    grid_fused.hip fused_mix_tile): per (mode, 16 realizations), two per k-step of each 16-pulsar tile, a lower-
    triangular factor's steps stopping at the tile's diagonal."""
    n_q = P if n_q is None else n_q
    steps = sum(-(-min(min(P, pt + 16) if lower else P, n_q) // 4) for pt in range(0, P, 16))
    return 2 * steps * nm * (R_pad // 16)


def kernel_avg_s(ctx, which):
    n, ms = ctx.kernel_stats(which)
    return ms / max(n, 1) / 1e3


def exact_roofline(ctx, capi, sim, seed, R, launches):
    """The exact fused kernel (path 3, k_synth_valu_seeded) on the same batch, timed with HIP events on the
    context stream after the main run: its FP64 rate against the MI355X FP64 peak (north-star target >= 50%)."""
    info = ctx.batch_info()
    old = ctx.get_option(capi.OPT_SYNTH_PATH)
    ctx.set_option(capi.OPT_SYNTH_PATH, 3)
    ctx.set_option(capi.OPT_PROFILE, 1)
    try:
        sim.synth(R, seed=seed, real0=0, to_host=False)  # warm (tile table)
        ctx.synchronize()
        ctx.reset_stats()
        for i in range(launches):
            sim.synth(R, seed=seed, real0=(i + 1) * R, to_host=False)
        ctx.synchronize()
        t = kernel_avg_s(ctx, capi.K_SYNTH)
    finally:
        ctx.set_option(capi.OPT_SYNTH_PATH, old)
        ctx.set_option(capi.OPT_PROFILE, 0)
    kernel = SYNTH_KERNELS[3][0]
    flops = 2.0 * info["K"] * info["n_toa"] * R
    achieved = flops / t / 1e12
    return {"kernel": kernel, "pipe": "fp64-valu", "launches": launches, "avg_launch_ms": t * 1e3,
            "flops_per_launch": flops, "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS, "write_GBps": 8.0 * info["n_toa"] * R / t / 1e9}


def isolated_grid(ctx, capi, sim, seed, R, launches):
    """The gridded kernels on the same batch with one stream (FPTA_OPT_OVERLAP 0), after the timed run: in the
    pipelined timed region the interpolation shares the CUs with the next block's draws and DFT, so its HIP-event
    time there includes that co-running work. Returns (interpolation, DFT) average launch seconds."""
    old = ctx.get_option(capi.OPT_OVERLAP)
    ctx.set_option(capi.OPT_OVERLAP, 0)
    ctx.set_option(capi.OPT_PROFILE, 1)
    try:
        sim.synth(R, seed=seed, real0=0, to_host=False)
        ctx.synchronize()
        ctx.reset_stats()
        for i in range(launches):
            sim.synth(R, seed=seed, real0=(i + 1) * R, to_host=False)
        ctx.synchronize()
        return kernel_avg_s(ctx, capi.K_SYNTH), kernel_avg_s(ctx, capi.K_GRID)
    finally:
        ctx.set_option(capi.OPT_OVERLAP, old)
        ctx.set_option(capi.OPT_PROFILE, 0)


def launch_ranks(n):
    """--gpus N > 1 without a launcher: run this command under torchrun as N rank processes (a child process;
    nothing here has touched a GPU) and return its exit status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: --gpus {n} without a launcher: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def hip_runtimes_mapped():
    """HIP runtime libraries mapped into this process (one expected: the library's ROCm 7.2 libamdhip64)."""
    try:
        with open("/proc/self/maps") as fh:
            return sorted({line.split()[-1] for line in fh if "libamdhip64" in line})
    except OSError:
        return None


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(world_env or 1)
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE)")
    refuse_debug_environment()
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator, RcclComm, RealizationComm, shard_bounds, simulate_sharded

    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = _capi.device_count()
    if args.dist_backend == "rccl":
        # one rank per GPU: a rank without its own device fails here instead of measuring fewer GPUs
        if local >= ndev:
            sys.exit(f"bench.py: rank with LOCAL_RANK {local} needs device {local}, but {ndev} device(s) are visible")
        device = local
    else:
        # gloo rehearsal: several ranks may share a card (local ranks wrap over the visible devices)
        device = local % max(ndev, 1)
    os.environ["FAKEPTA_AMD_DEVICE"] = str(device)  # the drop-in calls of build_array use the same card
    ctx = _capi.Context(device)
    if args.dist_backend == "gloo":
        comm = RealizationComm(backend="gloo", local_rank=device)
    elif world > 1:
        comm = RcclComm(ctx)
    else:
        comm = RealizationComm(world=1, rank=0, local_rank=device)  # one rank: no collective
    rank = comm.rank
    psrs = build_array(args.npsr, args.ntoa, args.config)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    info = ctx.batch_info()
    if args.path:
        ctx.set_option(_capi.OPT_SYNTH_PATH, args.path)
    if args.grid_mfma >= 0:
        ctx.set_option(_capi.OPT_GRID_MFMA, args.grid_mfma)
    if args.interp_ws >= 0:
        ctx.set_option(_capi.OPT_INTERP_WS, args.interp_ws)
    if args.overlap >= 0:
        ctx.set_option(_capi.OPT_OVERLAP, args.overlap)
    for kv in args.opt:
        name, val = kv.split("=")
        ctx.set_option(getattr(_capi, "OPT_" + name.upper()), int(val))

    if args.config == "c2":
        R = args.real
        for s in range(args.warmup):
            sim.synth(R, seed=args.seed, real0=(s * world + rank) * R, to_host=False)
        ctx.synchronize()
        ctx.set_option(_capi.OPT_PROFILE, 0 if args.no_kernel_events else 1)
        ctx.reset_stats()
        comm.barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        every = max(1, args.event_every)
        for s in range(args.steps):
            if not args.no_kernel_events and every > 1:
                ctx.set_option(_capi.OPT_PROFILE, 1 if s % every == 0 else 0)
            sim.synth(R, seed=args.seed, real0=((args.warmup + s) * world + rank) * R, to_host=False)
        ctx.synchronize()
        comm.barrier()
        dt = comm.max(time.perf_counter() - t0)
        n_samples_total = info["n_toa"] * R * args.steps * world
        sums = comm.gather_to_root(sim.checksums())  # last step's realizations, rank order = realization order
    else:
        R = args.c3_batch
        n_job = args.c3_real
        for s in range(args.warmup):  # warm every batch shape of the job (tile tables, grid plan, buffers)
            lo, hi = shard_bounds(n_job, rank, world)
            for first in range(lo, hi, R):
                sim.synth(min(R, hi - first), seed=args.seed, real0=first, to_host=False)
        ctx.synchronize()
        ctx.set_option(_capi.OPT_PROFILE, 1)
        ctx.reset_stats()
        comm.barrier()
        ctx.synchronize()
        t0 = time.perf_counter()
        for s in range(args.steps):
            sums = simulate_sharded(sim, n_job, seed=args.seed, real0=(args.warmup + s) * n_job, batch=R,
                                    comm=comm)
        ctx.synchronize()
        comm.barrier()
        dt = comm.max(time.perf_counter() - t0)
        n_samples_total = info["n_toa"] * n_job * args.steps

    ctx.set_option(_capi.OPT_PROFILE, 0)
    value = n_samples_total / dt
    synth_avg_s = kernel_avg_s(ctx, _capi.K_SYNTH) or float("nan")  # nan: --no-kernel-events
    synth_n = ctx.kernel_stats(_capi.K_SYNTH)[0]  # launches timed by events (--event-every)
    gi = ctx.batch_grid_info()
    path = gi["last_path"]
    # algorithmic bytes of one synthesis launch: 8 B per residual sample written; one launch
    # writes n_toa x R samples (c3: the job's batches averaged, the short last batch included)
    n_launch_real = R if args.config == "c2" else n_job / max(1, -(-shard_bounds(n_job, 0, world)[1] // R))
    out_bytes = 8.0 * info["n_toa"] * n_launch_real
    if path == 4:
        # the warp-specialised kernel serves plain blocks; fused-checksum blocks (c3) take the register kernel
        kernel = gi["interp_kernel"] or grid_interp_kernel(ctx.get_option(_capi.OPT_INTERP_WS), args.config != "c2",
                                                           -(-int(R) // 128) * 128)
        pipe = "fp64-mfma"
        traffic, traffic_src = pmc_traffic(kernel, info, R, args.traffic, GRID_LAYOUT)
        achieved = out_bytes / synth_avg_s / 1e9
        R_pad = -(-int(n_launch_real) // 128) * 128
        impl_bytes = out_bytes + 8.0 * gi["grid_vals"] * R_pad + gi["weight_bytes"]
        # the DFT launches of one step (pipelined C2: the per-pulsar DM grid signal's on a second side stream,
        # beside the other signals' on the first, FPTA_OPT_SIDE_SPLIT), their launch durations summed
        n_dft, dft_ms = ctx.kernel_stats(_capi.K_GRID)
        n_steps = args.steps if args.config == "c2" else max(n_dft, 1)
        grid_avg_s = dft_ms / 1e3 / n_steps
        dft_flops = 2.0 * gi["fma_dft"] * R_pad
        # grid signals with a per-pulsar member draw their coefficients inside the DFT (FPTA_OPT_DFT_GEN, C2)
        fused = kernel.startswith("k_grid_fused")
        mix_flops = (2048.0 * next_mix_mfmas(info["n_psr"], 30, R_pad)
                     if fused and args.config == "c2" and gi.get("next_mix_made") else 0.0)
        dft_kernel = ("inside " + kernel if fused else
                      "k_grid_dft_gen" if args.config == "c2" and ctx.get_option(_capi.OPT_DFT_GEN)
                      and gi["grid_mfma"] & 1 else GRID_DFT[bool(gi["grid_mfma"] & 1)])
        roofline = {"bound": "hbm", "pipe": pipe, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": kernel,
                    "algorithmic_bytes_per_launch": out_bytes, "avg_launch_ms": synth_avg_s * 1e3,
                    "event_launches": synth_n,
                    "traffic_over_algorithmic": (traffic / out_bytes) if traffic else None,
                    "traffic_source": traffic_src,
                    "implementation_bytes_per_launch": impl_bytes,
                    "interp_fp64_TFLOPs": 2.0 * gi["fma_interp_run"] * R_pad / synth_avg_s / 1e12,
                    # k_grid_fused also runs the block's DFTs on the same fp64 pipe (one launch, no DFT kernel): its
                    # interpolation + DFT MFMA FLOPs against the 78.6 TF FP64 peak beside the HBM fraction
                    # (+ the next block's GW mix when the launch made it: C2's HD GWB30, Cholesky factor)
                    "fp64_pipe": ({"flops_per_launch": 2.0 * (gi["fma_interp_run"] + gi["fma_dft"]) * R_pad + mix_flops,
                                   "next_mix_flops": mix_flops,
                                   "TFLOPs": (2.0 * (gi["fma_interp_run"] + gi["fma_dft"]) * R_pad + mix_flops)
                                   / synth_avg_s / 1e12,
                                   "frac": (2.0 * (gi["fma_interp_run"] + gi["fma_dft"]) * R_pad + mix_flops)
                                   / synth_avg_s / 1e12 / FP64_PEAK_TFLOPS} if fused else None),
                    "grid": {"width": gi["width"], "sigma": gi["sigma"], "err_bound": gi["err_bound"],
                             "signals": gi["signals"], "grid_signals": gi["grid_signals"],
                             "band_rows_per_chunk": gi["band_rows_per_chunk"]},
                    "dft": {"kernel": dft_kernel, "launches_per_step": n_dft / n_steps,
                            "co_running_span_ms_per_step": grid_avg_s * 1e3,
                            "note": ("the DFTs run inside the synthesis kernel (no DFT launch)" if fused else
                                     "HIP-event spans of one block's DFT launches on the side streams, beside the "
                                     "previous block's interpolation (not kernel durations; see isolated)"),
                            "flops_per_block": dft_flops}}
    else:
        # exact paths: FP64-bound, 2K FLOP per 8-byte sample (80 FLOP/B at K = 320)
        kernel, pipe = SYNTH_KERNELS[path]
        traffic, traffic_src = pmc_traffic(kernel, info, R, args.traffic)
        flops = 2.0 * info["K"] * info["n_toa"] * n_launch_real
        achieved = flops / synth_avg_s / 1e12
        roofline = {"bound": "mfma", "pipe": pipe, "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic, "kernel": kernel,
                    "traffic_source": traffic_src, "flops_per_launch": flops, "avg_launch_ms": synth_avg_s * 1e3,
                    "write_GBps": out_bytes / synth_avg_s / 1e9}

    if path == 4:
        # the HBM rate plain streaming stores reach on this part (torch fill of 6.5 GB, tools/store_rate.py): the
        # practical write ceiling beside the 8 TB/s spec the fraction above is taken against
        try:
            with open(os.path.join(ROOT, "profiles", "r03u_store_rate.json")) as fh:
                sr = json.load(fh)
            roofline["achievable_write"] = {"fill_GBps": sr["fill_TBps"] * 1e3,
                                            "copy_rw_GBps": sr["copy_TBps_read_plus_write"] * 1e3,
                                            "frac_of_fill": roofline["achieved"] / (sr["fill_TBps"] * 1e3),
                                            "source": "profiles/r03u_store_rate.json (tools/store_rate.py)"}
        except (OSError, ValueError, KeyError):
            pass
    if path == 4 and args.config == "c2" and args.exact_launches > 0:
        t_int, t_dft = isolated_grid(ctx, _capi, sim, args.seed, R, args.exact_launches)
        roofline["isolated"] = {"note": "same batch, one stream (no co-running draws / DFT), after the timed run",
                                "avg_launch_ms": t_int * 1e3, "achieved": out_bytes / t_int / 1e9,
                                "frac": out_bytes / t_int / 1e9 / HBM_PEAK_GBS, "dft_ms_per_block": t_dft * 1e3}
        if t_dft > 0:  # a layout whose DFT runs inside the synthesis kernel records no separate launch
            dft_tf = 2.0 * gi["fma_dft"] * (-(-R // 128) * 128) / t_dft / 1e12
            roofline["isolated"].update(dft_TFLOPs=dft_tf, dft_frac_fp64_peak=dft_tf / FP64_PEAK_TFLOPS)
    pcie = None
    if args.config == "c2" and args.exact_launches > 0:
        # PCIe-inclusive rate (never `value`): every step's block copied to a host numpy array
        sim.synth(R, seed=args.seed, real0=0, to_host=True)
        t0 = time.perf_counter()
        for i in range(2):
            sim.synth(R, seed=args.seed, real0=(i + 1) * R, to_host=True)
        dt_h = (time.perf_counter() - t0) / 2
        pcie = {"note": "block copied to pageable host memory every step (not the metric)",
                "ms_per_step": dt_h * 1e3, "samples_per_s": info["n_toa"] * R / dt_h,
                "host_GBps": 8.0 * info["n_toa"] * R / dt_h / 1e9}
    roofline_exact = None
    if args.config == "c2" and args.exact_launches > 0:
        roofline_exact = exact_roofline(ctx, _capi, sim, args.seed, R, args.exact_launches)

    if rank == 0:
        if args.config == "c2":
            workload = ("C2 (BASELINE configs[1]): %d psr x %d TOAs, RN30 + DM100(nu^-2) + HD GWB30, "
                        "%d realizations/GPU/step, Philox seed %d" % (args.npsr, args.ntoa, R, args.seed))
            scaling, per_key, per_val = "weak", "realizations_per_gpu", R
        else:
            workload = ("C3 (BASELINE configs[2]): %d psr x %d TOAs, HD GWB30 only, %d realizations per job "
                        "sharded over %d GPU(s) in batches of %d, checksums gathered to rank 0, Philox seed %d"
                        % (args.npsr, args.ntoa, n_job, world, R, args.seed))
            scaling, per_key, per_val = "strong", "realizations_per_job", n_job
        line = {
            "metric": METRIC, "value": value, "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": dt / args.steps * 1e3, "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload, "n_psr": args.npsr, "n_toa_total": info["n_toa"], "K": info["K"],
                       per_key: per_val, "parallelism": "realization-sharded x%d" % world},
            "synth_path": {1: "direct", 2: "mfma", 3: "valu-seeded", 4: "gridded"}.get(path, str(path)),
            "path_reason": gi["path_reason"] or None,
            "roofline": roofline,
            "roofline_exact": roofline_exact,
            "pcie_inclusive": pcie,
            "comm": {"backend": getattr(comm, "backend", "none") if world > 1 else "none (one rank)",
                     "hip_runtimes_mapped": hip_runtimes_mapped()},
            "checksum": float(np.sum(sums[:, 1])),
            "n_checksums": int(len(sums)),
        }
        if world == 1 and args.cpu_sample > 0:
            line["cpu_baseline"] = cpu_baseline(sim, psrs, args.cpu_sample, args.seed)
        else:
            line["cpu_baseline"] = None
        if world == 1 and args.config == "c2" and args.sub_configs:
            # the other BASELINE configs, each on its own context after the timed C2 region (value unchanged)
            from tools import bench_configs
            bench_configs.OPTS.extend(args.opt)
            line.update(bench_configs.sub_records())
        print(json.dumps(line), flush=True)
    ctx.close()
    comm.close()


if __name__ == "__main__":
    main()
