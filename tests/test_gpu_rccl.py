"""RCCL in the product's own process (reference loop that shards: correlated_noises.py:153-160).

The library links the system RCCL (ROCm 7.2, the kernels' HIP runtime) and exposes it two ways:
  * fpta_comm_* / fakepta_amd.batch.RcclComm: one process per GPU, the unique id exchanged over a plain TCP socket;
  * fpta_multi_synth with FPTA_GATHER_RCCL: one process driving several devices, ncclCommInitAll + one ncclGather
    of every device's checksums to device 0.
On a one-GPU box both run as one-rank communicators: the collectives execute (RCCL init, allreduce, gather) and
their results must equal the single-context stream bit for bit. The driver's N-GPU bench runs the same code with
one rank per GPU. A bench asked for more GPUs than the box has fails instead of measuring fewer, and a rank process
maps exactly one HIP runtime."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 99


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def small():
    from fakepta import correlated_noises as cn
    from fakepta import fake_pta as fp
    from fakepta_amd import _capi
    from fakepta_amd.batch import BatchSimulator
    ctx = _capi.Context(0)
    np.random.seed(3)
    psrs = fp.make_fake_array(npsrs=20, Tobs=10, ntoas=500, gaps=False, isotropic=True, toaerr=1e-7,
                              backends="NUPPI.1400", custom_model={"RN": 30, "DM": None, "Sv": None})
    cn.add_common_correlated_noise(psrs, orf="hd", log10_A=-15, gamma=13 / 3, components=30)
    sim = BatchSimulator(psrs, white=False, ctx=ctx)
    yield sim, ctx
    ctx.close()


def test_one_rank_rccl_comm(small):
    """RcclComm with one rank: socket rendezvous, ncclCommInitRank, allreduce-max and ncclGather; the sharded
    job's gathered checksums equal the single-context stream's."""
    from fakepta_amd.batch import RcclComm, simulate_sharded
    sim, ctx = small
    want = simulate_sharded(sim, 3000, seed=SEED, real0=5, batch=1024)
    comm = RcclComm(ctx, world=1, rank=0, addr="127.0.0.1", port=_free_port())
    try:
        assert comm.max(3.25) == 3.25
        comm.barrier()
        x = np.arange(12.0).reshape(6, 2)
        np.testing.assert_array_equal(comm.gather_to_root(x), x)
        got = simulate_sharded(sim, 3000, seed=SEED, real0=5, batch=1024, comm=comm)
        np.testing.assert_array_equal(got, want)
    finally:
        comm.close()


def test_multi_device_rccl_gather(small):
    """fpta_multi_synth with the RCCL gather (ncclCommInitAll over the listed devices, ncclGather to device 0)
    equals the single-context stream; duplicate devices cannot form a communicator and say so."""
    from fakepta_amd import _capi
    from fakepta_amd.batch import simulate_sharded
    sim, ctx = small
    want = simulate_sharded(sim, 2500, seed=SEED, real0=40, batch=1000)
    for devices, mode, route in (([0], _capi.GATHER_RCCL, _capi.GATHER_RCCL),
                                 ([0], _capi.GATHER_AUTO, _capi.GATHER_RCCL),
                                 ([0, 0], _capi.GATHER_AUTO, _capi.GATHER_HOST)):
        m = _capi.MultiContext(devices)
        try:
            m.set_toas(sim.offs, sim.toas, sim.freqs)
            for s in sim.segments:
                m.add_signal(s["kind"], s["f"], s["amp"], idx=s["idx"], L=s["L"], mask=s["mask"])
            m.set_gather(mode)
            np.testing.assert_array_equal(m.synth_checksums(SEED, 40, 2500, batch=1000), want)
            assert m.last_gather() == route
            np.testing.assert_array_equal(m.synth_checksums(SEED, 40, 2500, batch=700), want)  # comm reused
            if devices == [0, 0]:
                m.set_gather(_capi.GATHER_RCCL)
                with pytest.raises(_capi.FptaError, match="distinct devices"):
                    m.synth_checksums(SEED, 40, 2500, batch=1000)
        finally:
            m.close()


def _bench(args, timeout=110):
    env = {k: v for k, v in os.environ.items() if not k.startswith("FPTA_") and k not in ("WORLD_SIZE", "RANK",
                                                                                         "LOCAL_RANK")}
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_bench_rank_maps_one_hip_runtime():
    res = _bench(["--config", "c3", "--c3-real", "3000", "--c3-batch", "1024", "--steps", "1", "--warmup", "1",
                  "--cpu-sample", "0"])
    assert res.returncode == 0, res.stderr[-2000:]
    line = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][0])
    assert line["n_gpus"] == 1
    maps = line["comm"]["hip_runtimes_mapped"]
    assert len(maps) == 1 and "torch" not in maps[0], maps


def test_bench_more_gpus_than_the_box_fails():
    """bench.py --gpus N without a launcher starts N ranks; a rank without its own device exits non-zero (the job
    is not reported as a smaller one)."""
    from fakepta_amd import _capi
    n = _capi.device_count() + 1
    res = _bench(["--gpus", str(n), "--config", "c3", "--c3-real", "2000", "--steps", "1", "--warmup", "0",
                  "--cpu-sample", "0"])
    assert res.returncode != 0
    assert "needs device" in res.stderr
    assert not any(ln.startswith("{") for ln in res.stdout.splitlines())
