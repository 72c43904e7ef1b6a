"""Host logic of the multi-rank RCCL path, on the CPU (no GPU, no RCCL call).

* `_exchange_unique_id` (fakepta_amd/batch.py): the TCP rendezvous that hands rank 0's RCCL unique id to the other
  ranks of a one-process-per-GPU job, at world 3 with ranks starting in shuffled order, a stray
  connection, a rank that drops its connection before acknowledging, and both timeout paths.
* `RcclComm.gather_to_root`: the ragged padding / trimming around the library's fixed-size gather, with a stub
  communicator standing in for `_capi.Comm` (the reference gathers per-pulsar residual blocks of different lengths
  the same way: /root/reference/fakepta/correlated_noises.py:153-160 loops over the ragged array).
"""
import multiprocessing as mp
import random
import socket
import struct
import time

import numpy as np
import pytest

from fakepta_amd import batch as B

ID = bytes(range(128))


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, delay, q, timeout=20.0):
    time.sleep(delay)
    try:
        got = B._exchange_unique_id(rank, world, "127.0.0.1", port, lambda: ID, timeout, n_bytes=len(ID))
        q.put((rank, got))
    except Exception as e:  # reported to the parent
        q.put((rank, repr(e)))


def _run_world(world, delays, port, before_ranks=None):
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, delays[r], q)) for r in range(world)]
    for p in procs:
        p.start()
    if before_ranks is not None:
        before_ranks()
    out = dict(q.get(timeout=60) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    return out


def _connect_when_up(port, deadline=10.0):
    t0 = time.monotonic()
    while True:
        try:
            return socket.create_connection(("127.0.0.1", port), timeout=2.0)
        except OSError:
            if time.monotonic() - t0 > deadline:
                raise
            time.sleep(0.05)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_world3_shuffled_start_order(seed):
    """Every rank of a world-3 job gets rank 0's id, whichever order the ranks start in (rank 0 last included:
    the others retry until its socket listens)."""
    rng = random.Random(seed)
    delays = [rng.uniform(0.0, 0.8) for _ in range(3)]
    out = _run_world(3, delays, _free_port())
    assert out == {0: ID, 1: ID, 2: ID}


def test_stray_and_dropped_connections_use_no_slot():
    """A connection with a wrong magic, one with an out-of-range rank, and a valid rank-2 hello that closes before
    acknowledging are all served or refused without counting: the real rank 1 and rank 2 still get the id and rank 0
    returns only after both acknowledged."""
    port = _free_port()

    def strays():
        c = _connect_when_up(port)
        c.sendall(b"HTTP")  # wrong magic, then nothing
        c.close()
        c = _connect_when_up(port)
        c.sendall(B._RDZV_MAGIC + struct.pack("<I", 7))  # rank outside the world
        c.close()
        c = _connect_when_up(port)
        c.sendall(B._RDZV_MAGIC + struct.pack("<I", 2))  # a rank that fails after connecting
        c.recv(16)
        c.close()

    out = _run_world(3, [0.0, 1.0, 1.5], port, before_ranks=strays)
    assert out == {0: ID, 1: ID, 2: ID}


def test_rank0_times_out_on_a_missing_rank():
    port = _free_port()
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_rank_main, args=(1, 3, port, 0.0, q))
    p.start()
    t0 = time.monotonic()
    with pytest.raises(TimeoutError, match=r"ranks \[2\]"):
        B._exchange_unique_id(0, 3, "127.0.0.1", port, lambda: ID, 2.0, n_bytes=len(ID))
    assert time.monotonic() - t0 < 10.0
    assert q.get(timeout=30) == (1, ID)
    p.join(timeout=30)


def test_rank_times_out_without_rank0():
    t0 = time.monotonic()
    with pytest.raises(TimeoutError, match="no RCCL rendezvous"):
        B._exchange_unique_id(2, 3, "127.0.0.1", _free_port(), lambda: ID, 1.0, n_bytes=len(ID))
    assert time.monotonic() - t0 < 10.0


def test_rank0_refuses_a_wrong_size_id():
    with pytest.raises(ValueError, match="unique id"):
        B._exchange_unique_id(0, 2, "127.0.0.1", _free_port(), lambda: ID[:10], 1.0, n_bytes=len(ID))


class _StubComm:
    """Stands in for _capi.Comm.gather: rank 0 receives every rank's [n_max, ...] block stacked in rank order."""

    def __init__(self, blocks, rank):
        self.blocks, self.rank = blocks, rank

    def gather(self, pad):
        self.blocks[self.rank] = pad.copy()
        return np.stack(self.blocks) if self.rank == 0 else None


@pytest.mark.parametrize("sizes", [[5, 5, 5], [4, 3, 3], [0, 2, 1], [7]])
def test_rccl_gather_pads_and_trims_ragged_shards(sizes):
    """gather_to_root pads each rank's rows to the largest shard for the fixed-size collective and rank 0 trims them
    back: the result is every rank's rows in rank order, nothing else."""
    world = len(sizes)
    rng = np.random.default_rng(len(sizes) + sum(sizes))
    shards = [rng.normal(size=(n, 2)) for n in sizes]
    blocks = [None] * world
    got = {}
    for r in reversed(range(world)):  # rank 0 last: the stub gathers the others' blocks first
        comm = object.__new__(B.RcclComm)
        comm.world, comm.rank, comm.comm = world, r, _StubComm(blocks, r)
        got[r] = comm.gather_to_root(shards[r], sizes)
    for r in range(1, world):
        assert got[r] is None
    np.testing.assert_array_equal(got[0], np.concatenate(shards))
    assert all(b.shape == (max(sizes), 2) for b in blocks)
