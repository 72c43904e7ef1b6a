"""Two ranks on one card (torch.distributed, gloo) against one rank: the C3 job sharded by simulate_sharded gathers
the same per-realization checksums to rank 0 (the driver's 2/4/8-GPU runs use RCCL with one rank
per GPU). bench.py prints rank 0's line; its checksum is the sum over the gathered realizations in global order,
so it must be bit-identical to the single-rank job's."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--config", "c3", "--c3-real", "10000", "--c3-batch", "4096", "--steps", "1", "--warmup", "1",
        "--cpu-sample", "0", "--dist-backend", "gloo"]


def _line(cmd):
    env = {k: v for k, v in os.environ.items() if not k.startswith("FPTA_")}
    env["MASTER_ADDR"] = "127.0.0.1"
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]
    return json.loads(lines[0])


def test_two_rank_c3_checksums_match_one_rank():
    one = _line([sys.executable, "bench.py"] + ARGS)
    two = _line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", "29531", "bench.py", "--gpus", "2"] + ARGS)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["n_checksums"] == two["n_checksums"] == 10000
    assert one["checksum"] == two["checksum"]


def test_two_rank_c2_steps_match_one_rank():
    """C2 on two ranks (gloo, one card): rank g's step s draws realizations ((W + s) 2 + g) R .. + R, so its blocks
    advance at a stride of two blocks (the library's next-block mix follows that stride, FPTA_OPT_FUSED_NEXT_MIX);
    the last step's realizations of both ranks, gathered in rank order, are one rank's last step at 2R realizations
    per step: the same checksums, bit for bit."""
    args = ["--steps", "4", "--warmup", "2", "--cpu-sample", "0", "--sub-configs", "0", "--exact-launches", "0",
            "--dist-backend", "gloo"]
    one = _line([sys.executable, "bench.py", "--real", "256"] + args)
    two = _line([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                 "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py", "--gpus", "2", "--real", "128"]
                + args)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert one["n_checksums"] == two["n_checksums"] == 256
    assert one["checksum"] == two["checksum"]
