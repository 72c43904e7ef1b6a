"""Batched realizations: many independent draws of an array's noise model on one MI355X.

The reference produces one realization per Python call (make_fake_array / add_* /
add_common_correlated_noise, a loop over pulsars and modes). BatchSimulator takes the noise
model an array already carries (each Pulsar's signal_model and noisedict, as left by
make_fake_array or the add_* injectors) and re-draws it R times on the device:

    Philox4x32-10 draws -> ORF mixing -> fused basis/contraction -> white/ECORR

Realization r of seed s is the same whatever the batch split or number of GPUs (the Philox
counter carries the global realization index), so realizations shard across ranks with no
data-path collective. The draws are not numpy's MT19937 stream (SURVEY.md §7 'RNG parity');
the oracle (oracle/fakepta_oracle.py: batch_synth) restates the exact semantics.
"""
import numpy as np

from . import _capi
from fakepta.correlated_noises import orf_factor, orf_matrix

GP_NAMES = ("red_noise", "dm_gp", "chrom_gp")


def _df(f):
    return np.diff(np.append(0.0, f))


def _n_modes(sm):
    """Modes a stored signal carries: its coefficient pairs, at most len(f) (reconstruct_signal's zip,
    fake_pta.py:543; a common signal stores `components` pairs on a longer f_psd, correlated_noises.py:140-143)."""
    n = len(sm["f"])
    return min(n, np.shape(sm["fourier"])[1]) if "fourier" in sm else n


def batch_factor(orf_mat):
    """Square root of the ORF for batched draws: the lower Cholesky factor when the ORF is
    positive definite (HD, curn: triangular mixing on device, half the FLOPs), otherwise the SVD
    factor numpy's multivariate_normal uses (singular monopole / dipole ORFs). Any L with
    L L^T = ORF gives the reference's distribution; the drop-in path keeps numpy's exact factor."""
    try:
        return np.ascontiguousarray(np.linalg.cholesky(orf_mat))
    except np.linalg.LinAlgError:
        # singular ORF (monopole: rank 1, dipole: rank 3): the SVD factor with the directions of numerically zero
        # variance (singular values <= 1e-12 of the largest, i.e. rounding noise of a rank-r matrix) set to exact
        # zeros, so the device mixes (and draws normals for) only the first r columns; L L^T changes by <= 1e-12
        # relative
        _, s, _ = np.linalg.svd(orf_mat)
        L = orf_factor(orf_mat)
        L[:, s <= 1e-12 * s[0]] = 0.0
        return np.ascontiguousarray(L)


class BatchSimulator:
    """Device-resident noise model of an array of Pulsar objects.

    signals: names to include (default: every GP signal found in the pulsars' signal_model:
             red_noise, dm_gp, chrom_gp, '*system_noise*' and '*common*').
    white:   include EFAC/EQUAD white noise from each pulsar's noisedict.
    ecorr:   include ECORR epochs (ENTERPRISE convention 10^(2 log10_ecorr)).
    """

    def __init__(self, psrs, signals=None, white=True, ecorr=False, device=None, ctx=None):
        self.psrs = psrs
        self.ctx = ctx if ctx is not None else _capi.get_context(device)
        self.offs = np.concatenate([[0], np.cumsum([len(p.toas) for p in psrs])]).astype(np.int64)
        self.toas = np.concatenate([p.toas for p in psrs])
        self.freqs = np.concatenate([p.freqs for p in psrs])
        self.ctx.batch_set_toas(self.offs, self.toas, self.freqs)
        self.segments = []  # (name, kind, f, amp, idx, L, mask) — host copy for checking/reporting
        names = signals
        if names is None:
            names = []
            for p in psrs:
                for s in p.signal_model:
                    if s not in names and (s in GP_NAMES or "common" in s or "system_noise" in s):
                        names.append(s)
        for name in names:
            self._add_named(name)
        if white or ecorr:
            self._set_white(white, ecorr)

    # ------------------------------------------------------------------ layout building
    def _add_named(self, name):
        P = len(self.psrs)
        have = [p for p in self.psrs if name in p.signal_model]
        if not have:
            raise KeyError(f"no pulsar carries signal {name!r}")
        sm0 = have[0].signal_model[name]
        if "common" in name:
            n = _n_modes(sm0)
            f = np.asarray(sm0["f"], float)
            amp = np.sqrt(np.asarray(sm0["psd"], float) * _df(f))[:n]
            f = f[:n]
            L = batch_factor(orf_matrix(self.psrs, sm0["orf"], sm0.get("hmap")))
            self.add_signal(name, 1, f, amp, idx=float(sm0["idx"]), L=L)
            return
        nm = max(_n_modes(p.signal_model[name]) for p in have)
        f = np.zeros((P, nm))
        amp = np.zeros((P, nm))
        mask = None
        for i, p in enumerate(self.psrs):
            if name in p.signal_model:
                sm = p.signal_model[name]
                n = _n_modes(sm)
                fi = np.asarray(sm["f"], float)
                amp[i, :n] = np.sqrt(np.asarray(sm["psd"], float) * _df(fi))[:n]
                fi = fi[:n]
                f[i, :n] = fi
                if len(fi) < nm:  # continue the grid with zero-amplitude modes
                    step = fi[0] if len(fi) else 1.0
                    f[i, len(fi):] = fi[-1] + step * np.arange(1, nm - len(fi) + 1)
            else:
                f[i] = np.arange(1, nm + 1) / max(np.ptp(p.toas), 1.0)
        idx = float(sm0["idx"])
        if "system_noise" in name:
            backend = name.split("system_noise_")[1]
            mask = np.concatenate([p.backend_flags == backend for p in self.psrs]).astype(np.uint8)
            idx = 0.0
        self.add_signal(name, 0, f, amp, idx=idx, mask=mask)

    def add_signal(self, name, kind, f, amp, idx=0.0, freqf=1400.0, L=None, mask=None):
        """Add one GP: kind 0 per-pulsar (f, amp [P, N]) or kind 1 common (f, amp [N], L [P, P])."""
        sid = self.ctx.batch_add_signal(kind, f, amp, idx=idx, freqf=freqf, L=L, mask=mask)
        self.segments.append(dict(name=name, kind=kind, f=np.asarray(f, float), amp=np.asarray(amp, float),
                                  idx=float(idx), freqf=float(freqf), L=L, mask=mask, id=sid))
        return sid

    def _set_white(self, white, ecorr):
        sigma = np.concatenate([p._white_sigma2() ** 0.5 for p in self.psrs]) if white else None
        blocks, esig = [], []
        if ecorr:
            for i, p in enumerate(self.psrs):
                for b in p.backends:
                    key = f"{p.name}_{b}_log10_ecorr"
                    if key not in p.noisedict:
                        continue
                    for q in p.ecorr_blocks(backends=[b]):
                        blocks.append(q + self.offs[i])
                        esig.append(10 ** p.noisedict[key])
        self.sigma = sigma
        self.blocks = blocks
        self.ecorr_sigma = np.array(esig)
        self.ctx.batch_set_white(sigma, blocks if blocks else None, self.ecorr_sigma if blocks else None)

    # ------------------------------------------------------------------ running
    @property
    def n_toa(self):
        return int(self.offs[-1])

    def synth(self, n_real, seed=0, real0=0, to_host=True, coeffs=False):
        """Realizations real0 .. real0+n_real-1: returns [n_real, n_toa] (host) or None (device only)."""
        return self.ctx.batch_synth(seed, real0, n_real, to_host=to_host, coeffs=coeffs)

    def synth_from_z(self, z):
        """Validation mode: z [n_real, n_seg, P, N_max, 2] standard normals (cos, sin)."""
        return self.ctx.batch_synth_from_z(z)

    def correlations(self, normalized=True):
        """Mean over the last block's realizations of the zero-lag cross-correlation matrix
        dot(res_a, res_b)/n (correlated_noises.py:14-19), normalized per realization by the
        auto-correlations if `normalized`. Computed on device; pulsars must share the TOA count."""
        _, _, R = self.ctx.batch_device_out()
        return self.ctx.batch_correlations(2 if normalized else 1) / R

    def hd_curve(self, bins=10, estimator="ratio", return_counts=False):
        """(mean, std, bin centres) of the pairwise correlations against angular separation
        (correlated_noises.py:21-47) for the last block. estimator "ratio": mean cross-power over
        sqrt(mean auto-powers) (consistent); "per_realization": mean of per-realization normalized
        correlations (biased toward 0 by O(1/n_eff) for red processes). A bin with no pulsar pair is NaN,
        as the reference's bin_curve gives, but without NumPy's empty-slice warnings; return_counts=True
        appends the number of pairs per bin so callers can mask the empty ones."""
        if estimator == "ratio":
            C = self.correlations(normalized=False)
            d = np.sqrt(np.diag(C))
            C = C / np.outer(d, d)
        else:
            C = self.correlations(normalized=True)
        pos = np.array([p.pos for p in self.psrs])
        iu = np.triu_indices(len(self.psrs), 1)
        angles = np.arccos(np.clip(pos @ pos.T, -1.0, 1.0))[iu]
        corrs = C[iu]
        edges = np.linspace(0., np.pi, bins + 1)
        centres = edges[:-1] + 0.5 * (edges[1] - edges[0])
        mean, std, counts = np.full(bins, np.nan), np.full(bins, np.nan), np.zeros(bins, dtype=np.int64)
        for b, (lo, hi) in enumerate(zip(edges[:-1], edges[1:])):
            sel = corrs[(angles > lo) & (angles < hi)]  # open bins, as correlated_noises.py:36-47
            counts[b] = len(sel)
            if len(sel):
                mean[b], std[b] = np.mean(sel), np.std(sel)
        return (mean, std, centres, counts) if return_counts else (mean, std, centres)

    def checksums(self):
        """Per-realization (sum, sum of squares) of the last block, computed on device."""
        return self.ctx.batch_checksums()

    def split(self, block):
        """[n_real, n_toa] -> list of per-pulsar [n_real, n_p] views."""
        return [block[..., self.offs[i]:self.offs[i + 1]] for i in range(len(self.psrs))]


def simulate_batch(psrs, n_real, seed=0, real0=0, signals=None, white=True, ecorr=False, device=None):
    """One-call convenience: [n_real, n_toa_total] residual realizations of the array's noise model."""
    return BatchSimulator(psrs, signals=signals, white=white, ecorr=ecorr, device=device).synth(
        n_real, seed=seed, real0=real0)


# ----------------------------------------------------------------------------- multi-GPU (one process per GPU)
def shard_bounds(n_real, rank, world):
    """Realizations [start, end) of rank `rank` of `world` for a job of n_real (rank g owns
    [g R / G, (g + 1) R / G)); contiguous, disjoint, covering, sizes differing by at most one."""
    return rank * n_real // world, (rank + 1) * n_real // world


class RealizationComm:
    """torch.distributed plumbing of a realization-sharded job: one process per rank launched by torchrun
    (WORLD_SIZE / RANK / LOCAL_RANK from the environment), backend "gloo" (CPU tests, rehearsals of several ranks
    on one card) or "nccl". GPU jobs use RcclComm instead: torch's "nccl" backend would bring torch's own HIP
    runtime and RCCL (ROCm 7.0) into a process whose kernels run on the library's (ROCm 7.2). The data path has no
    collective: only the timing barrier, a max-reduce of the elapsed time and the gather of per-realization
    checksums to rank 0 go through it."""

    def __init__(self, backend="nccl", world=None, rank=None, local_rank=None):
        import os
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else int(world)
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0")) if local_rank is None else int(local_rank)
        self.backend = backend
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            self.torch = torch
            if backend == "nccl":
                ndev = torch.cuda.device_count()
                torch.cuda.set_device(self.local_rank % max(ndev, 1))
                self.device = torch.device("cuda", torch.cuda.current_device())
            else:
                self.device = torch.device("cpu")
            if not dist.is_initialized():
                dist.init_process_group(backend=backend)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, x):
        """max over ranks of a float (the job time is the slowest rank's)."""
        if not self.dist:
            return float(x)
        t = self.torch.tensor([float(x)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather_to_root(self, arr, rows_per_rank=None):
        """Rank 0 receives every rank's `arr` ([n_g, ...] float64; n_g may differ by rank) concatenated in
        rank order; other ranks get None. rows_per_rank: list of n_g (known to every rank); arrays are padded
        to the largest n_g for the collective and trimmed on rank 0."""
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        if not self.dist:
            return arr.copy()
        if rows_per_rank is None:
            rows_per_rank = [arr.shape[0]] * self.world
        n_max = max(rows_per_rank)
        pad = np.zeros((n_max,) + arr.shape[1:])
        pad[:arr.shape[0]] = arr
        t = self.torch.from_numpy(pad).to(self.device)
        bufs = [self.torch.empty_like(t) for _ in range(self.world)] if self.rank == 0 else None
        self.dist.gather(t, gather_list=bufs, dst=0)
        if self.rank != 0:
            return None
        return np.concatenate([b.cpu().numpy()[:n] for b, n in zip(bufs, rows_per_rank)])

    def close(self):
        if self.dist and self.dist.is_initialized():
            self.dist.destroy_process_group()
        self.dist = None


_RDZV_MAGIC = b"FPTA"


def _recv_exact(conn, n):
    buf = b""
    while len(buf) < n:
        chunk = conn.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous connection closed early")
        buf += chunk
    return buf


def _exchange_unique_id(rank, world, addr, port, make_id, timeout, n_bytes=None):
    """Rank 0 makes the RCCL unique id and serves it to ranks 1 .. world - 1 over one TCP socket at (addr, port);
    the other ranks connect (retrying until `timeout`) and read its bytes. Plain sockets: no torch import, so the
    rank process maps one HIP runtime (the library's).

    Protocol: a rank sends b"FPTA" + its rank (uint32 little-endian), reads the id, answers b"A" and returns only once
    rank 0 has confirmed with b"K". Rank 0 counts a rank as served after reading its b"A" and sending b"K", and keeps
    accepting until every rank 1 .. world - 1 is served: a peer with a wrong magic or rank, or one that drops the
    connection before its acknowledgement, uses up no slot; a rank whose acknowledgement rank 0 did not read (timeout,
    reset) gets no confirmation, connects again and is served again. Either side raises TimeoutError past `timeout`
    seconds."""
    import socket
    import struct
    import time as _time
    n = _capi.COMM_ID_BYTES if n_bytes is None else int(n_bytes)
    deadline = _time.monotonic() + timeout
    if rank == 0:
        uid = make_id()
        if len(uid) != n:
            raise ValueError(f"unique id of {len(uid)} bytes, expected {n}")
        pending = set(range(1, world))
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as srv:
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(max(world, 8))
            while pending:
                left = deadline - _time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"rank 0: RCCL rendezvous at {addr}:{port}: ranks {sorted(pending)} did not "
                                       f"check in within {timeout} s")
                srv.settimeout(left)
                try:
                    conn, _ = srv.accept()
                except socket.timeout:
                    continue
                with conn:
                    try:
                        conn.settimeout(min(5.0, max(deadline - _time.monotonic(), 0.1)))
                        hello = _recv_exact(conn, 8)
                        peer = struct.unpack("<I", hello[4:])[0]
                        if hello[:4] != _RDZV_MAGIC or not 1 <= peer < world:
                            continue  # a stray or foreign connection: no slot used
                        conn.sendall(uid)
                        if _recv_exact(conn, 1) == b"A":
                            conn.sendall(b"K")
                            pending.discard(peer)
                    except OSError:
                        continue  # no confirmation sent: the peer connects again
        return uid
    hello = _RDZV_MAGIC + struct.pack("<I", rank)
    while True:
        try:
            with socket.create_connection((addr, port), timeout=5.0) as conn:
                conn.sendall(hello)
                buf = _recv_exact(conn, n)
                conn.sendall(b"A")
                if _recv_exact(conn, 1) == b"K":  # rank 0 recorded this rank
                    return buf
        except OSError:
            pass  # no rank 0 yet, or no confirmation: connect again
        if _time.monotonic() > deadline:
            raise TimeoutError(f"rank {rank}: no RCCL rendezvous at {addr}:{port} within {timeout} s")
        _time.sleep(0.2)


class RcclComm:
    """RCCL over xGMI for a realization-sharded job with one process per GPU, launched by
    torchrun (WORLD_SIZE / RANK / MASTER_ADDR / MASTER_PORT from the environment). The communicator is the
    library's own (fpta_comm_*: the system RCCL on the kernels' HIP runtime), on the rank's context and stream;
    torch is never imported, so each rank maps one HIP runtime. Rank 0's 128-byte unique id reaches the others
    over a TCP socket at (MASTER_ADDR, MASTER_PORT + 1) (torchrun's own store listens on MASTER_PORT;
    FAKEPTA_AMD_RDZV_PORT overrides). Same interface as RealizationComm: barrier, max, gather_to_root, close."""

    backend = "rccl"

    def __init__(self, ctx, world=None, rank=None, addr=None, port=None, timeout=120.0):
        import os
        self.world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else int(world)
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else int(rank)
        self.local_rank = ctx.device
        self.ctx = ctx
        addr = addr or os.environ.get("MASTER_ADDR", "127.0.0.1")
        if port is None:
            port = int(os.environ.get("FAKEPTA_AMD_RDZV_PORT", int(os.environ.get("MASTER_PORT", "29500")) + 1))
        uid = _exchange_unique_id(self.rank, self.world, addr, int(port), _capi.Comm.unique_id, timeout)
        self.comm = _capi.Comm(ctx, self.world, self.rank, uid)

    def barrier(self):
        self.comm.max(0.0)

    def max(self, x):
        """max over ranks of a float (the job time is the slowest rank's)."""
        return self.comm.max(x)

    def gather_to_root(self, arr, rows_per_rank=None):
        """As RealizationComm.gather_to_root: rank 0 gets every rank's rows in rank order (padded to the largest
        count for the collective, trimmed here), the other ranks None."""
        arr = np.ascontiguousarray(arr, dtype=np.float64)
        if rows_per_rank is None:
            rows_per_rank = [arr.shape[0]] * self.world
        n_max = max(rows_per_rank)
        pad = np.zeros((n_max,) + arr.shape[1:])
        pad[:arr.shape[0]] = arr
        got = self.comm.gather(pad)
        if got is None:
            return None
        return np.concatenate([got[g, :n] for g, n in enumerate(rows_per_rank)])

    def close(self):
        if getattr(self, "comm", None) is not None:
            self.comm.close()
            self.comm = None


def simulate_sharded(sim, n_real, seed=0, real0=0, batch=4096, comm=None, on_batch=None):
    """Realizations real0 .. real0 + n_real - 1 of `sim`'s noise model over every rank of `comm`.

    Rank g of G synthesizes its shard [real0 + g n / G, real0 + (g + 1) n / G) (shard_bounds) in batches of
    <= `batch` realizations on its own GPU, keeps each batch resident on the device (on_batch(sim, first, n)
    may consume it there: correlations, downloads) and computes per-realization checksums on the device.
    Rank 0 receives all checksums, in global realization order: returns [n_real, 2] (sum, sum of squares)
    on rank 0 and None on the other ranks. TOAs, tables and the ORF factor are replicated (each rank builds
    its own BatchSimulator); realization r is bit-identical whatever G and `batch` are (Philox counters carry
    the global index), which tests/test_dist_gloo.py and tests/test_gpu_c3.py check.

    sim: BatchSimulator (or any object with synth(n, seed=, real0=, to_host=False) and checksums()).
    comm: RcclComm (GPU ranks) or RealizationComm (gloo; default: a single-rank job)."""
    comm = comm if comm is not None else RealizationComm(world=1, rank=0, local_rank=0)
    G = comm.world
    lo, hi = shard_bounds(n_real, comm.rank, G)
    sums = np.empty((hi - lo, 2))
    # checksums from the gridded interpolation's partial sums (FPTA_OPT_FUSE_CHECKSUMS): no second pass over
    # each resident block;
    # each rank's context's own settings are restored afterwards. The synthesis path is chosen once for the job
    # (FPTA_OPT_MFMA_MIN_REAL 1): a tail batch below the default threshold would otherwise take the direct path, and
    # its realizations would depend on the batch split and the number of ranks
    ctx = getattr(sim, "ctx", None)
    fuse = min_real = None
    if ctx is not None:
        from fakepta_amd import _capi
        fuse = ctx.get_option(_capi.OPT_FUSE_CHECKSUMS)
        min_real = ctx.get_option(_capi.OPT_MFMA_MIN_REAL)
        ctx.set_option(_capi.OPT_FUSE_CHECKSUMS, 1)
        ctx.set_option(_capi.OPT_MFMA_MIN_REAL, 1)
    try:
        if ctx is not None and on_batch is None and hi > lo:
            # no per-batch consumer: the whole shard streams inside the library, batches back to back
            sums[:] = ctx.batch_synth_checksums(seed, real0 + lo, hi - lo, batch)
        for first in range(lo, hi, batch) if ctx is None or on_batch is not None else ():
            n = min(batch, hi - first)
            sim.synth(n, seed=seed, real0=real0 + first, to_host=False)
            if on_batch is not None:
                on_batch(sim, real0 + first, n)
            sums[first - lo:first - lo + n] = sim.checksums()
    finally:
        if fuse is not None:
            ctx.set_option(_capi.OPT_FUSE_CHECKSUMS, fuse)
            ctx.set_option(_capi.OPT_MFMA_MIN_REAL, min_real)
    sizes = [shard_bounds(n_real, g, G)[1] - shard_bounds(n_real, g, G)[0] for g in range(G)]
    return comm.gather_to_root(sums, sizes)
