"""Multi-rank product path on CPU (gloo, world size 2 and 4): fakepta_amd.batch.simulate_sharded shards a
job's realizations over the ranks, streams each shard in batches and gathers the per-realization checksums
to rank 0 in global order; RealizationComm's max-reduce and gather. The GPU synthesis is replaced by a CPU
stand-in whose checksum of realization g is a function of g alone (the oracle's Philox white-noise stream),
so the gathered result must equal a single-rank run bit for bit. No GPU involved."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class StandInSim:
    """synth()/checksums() of a BatchSimulator, computed on the CPU from the global realization index."""

    def __init__(self, n_toa=37):
        self.n_toa = n_toa
        self.calls = []
        self._block = None

    def synth(self, n_real, seed=0, real0=0, to_host=True):
        from oracle import fakepta_oracle as O
        self.calls.append((real0, n_real))
        self._block = O.white_normals_rpairs(seed, np.arange(real0, real0 + n_real), self.n_toa)
        return self._block if to_host else None

    def checksums(self):
        return np.stack([self._block.sum(1), (self._block ** 2).sum(1)], 1)


def _job(comm, n_real, seed, real0, batch):
    from fakepta_amd.batch import simulate_sharded
    sim = StandInSim()
    sums = simulate_sharded(sim, n_real, seed=seed, real0=real0, batch=batch, comm=comm)
    return sums, sim.calls


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from fakepta_amd.batch import RealizationComm
    comm = RealizationComm(backend="gloo")
    t = comm.max(0.5 + rank)
    ragged = comm.gather_to_root(np.full((rank + 1, 2), float(rank)), rows_per_rank=[g + 1 for g in range(world)])
    out = []
    for n_real, batch in ((1003, 100), (64, 4096), (5, 2)):
        out.append(_job(comm, n_real, seed=77, real0=1000 + n_real, batch=batch))
    comm.barrier()
    comm.close()
    q.put((rank, t, None if ragged is None else ragged.tolist(),
           [(None if s is None else s.tolist(), c) for s, c in out]))


@pytest.mark.parametrize("world", [2, 4])
def test_simulate_sharded_gather_to_root(world):
    from fakepta_amd.batch import RealizationComm, shard_bounds
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # max over ranks; ragged gather arrives on rank 0 only, in rank order
    assert all(abs(r[1] - (0.5 + world - 1)) < 1e-12 for r in res)
    assert all(r[2] is None for r in res[1:])
    g = np.array(res[0][2])
    assert g.shape == (world * (world + 1) // 2, 2)
    assert list(g[:, 0]) == [float(k) for k in range(world) for _ in range(k + 1)]
    single = RealizationComm(world=1, rank=0, local_rank=0)
    for j, (n_real, batch) in enumerate(((1003, 100), (64, 4096), (5, 2))):
        want, _ = _job(single, n_real, seed=77, real0=1000 + n_real, batch=batch)
        got = np.array(res[0][3][j][0])
        np.testing.assert_array_equal(got, want)  # bit-identical to the single-rank job, global order
        assert all(r[3][j][0] is None for r in res[1:])
        # each rank synthesized exactly its contiguous shard, in batches of <= batch
        for rank in range(world):
            lo, hi = shard_bounds(n_real, rank, world)
            calls = res[rank][3][j][1]
            covered = [i for r0, n in calls for i in range(r0, r0 + n)]
            assert covered == list(range(1000 + n_real + lo, 1000 + n_real + hi))
            assert all(n <= batch for _, n in calls)


def test_shard_bounds_partition():
    from fakepta_amd.batch import shard_bounds
    for n in (0, 1, 7, 100000, 100003):
        for world in (1, 2, 3, 4, 8):
            b = [shard_bounds(n, g, world) for g in range(world)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[g][1] == b[g + 1][0] for g in range(world - 1))
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 1
