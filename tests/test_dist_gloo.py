"""Multi-rank logic of bench.py on CPU (gloo, world size 2 and 4): realization sharding, the
max-over-ranks timing reduction and the checksum all-gather. No GPU involved."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import bench
    comm = bench.Comm(world, rank, rank, backend="gloo")
    R = 1024
    owned = [bench.shard_range(R, rank, world, step) for step in range(3)]
    t = comm.max(0.5 + rank)
    sums = np.full((4, 2), float(rank))
    allsums = comm.gather(sums)
    comm.barrier()
    comm.close()
    q.put((rank, owned, t, allsums.tolist()))


@pytest.mark.parametrize("world", [2, 4])
def test_sharding_reduction_gather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    # every realization index of every step is owned by exactly one rank, contiguous per rank
    for step in range(3):
        starts = sorted(r[1][step][0] for r in res)
        assert starts == [(step * world + g) * 1024 for g in range(world)]
    allidx = sorted(i for r in res for (s0, n) in r[1] for i in range(s0, s0 + n))
    assert allidx == list(range(3 * world * 1024))
    # max over ranks and gather in rank order
    assert all(abs(r[2] - (0.5 + world - 1)) < 1e-12 for r in res)
    for r in res:
        g = np.array(r[3])
        assert g.shape == (world, 4, 2)
        assert [g[k, 0, 0] for k in range(world)] == [float(k) for k in range(world)]
