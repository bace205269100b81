"""GPU: the RCCL (``nccl`` backend) path on the box's one GPU.

A world-size-1 group under ``torch.distributed.run`` (127.0.0.1) initialised exactly as bench.py
and the C5 driver do (``distributed.init_from_env``, ``device_id`` bound): the collectives run on
device tensors through RCCL even with a single rank (``all_reduce_sum`` has no world-size-1
shortcut), and the distributed loss / gradient / forward sweep equal the single-process ones.
Then bench.py itself under the launcher: its JSON reports the nccl backend and the one all-reduce
per step.  (N > 1 over RCCL needs one GPU per rank: the driver's multi-GPU runs.)
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun(args, env):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port())] + args
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_rccl_world_size_one_collectives():
    env = {k: v for k, v in os.environ.items() if k not in ("PFR_DIST_BACKEND", "PFR_BENCH_ONE_DEVICE")}
    out = _torchrun(["tests/_nccl_worker.py"], env)
    assert out["backend"] == "nccl" and out["world"] == 1
    # one all_reduce_sum of the test tensor, one per loss evaluation, one all-gather of fr
    assert out["collectives"] >= 3
    assert out["loss_rel"] < 1e-13 and out["grad_rel"] < 1e-12 and out["fr_rel"] < 1e-13


@pytest.mark.timeout(300)
def test_bench_under_launcher_uses_rccl():
    env = {k: v for k, v in os.environ.items() if k not in ("PFR_DIST_BACKEND", "PFR_BENCH_ONE_DEVICE")}
    out = _torchrun(["bench.py", "--gpus", "1", "--ny", "6", "--freqs", "512", "--steps", "2", "--warmup", "1",
                     "--no-cpu-baseline", "--chunk", "256"], env)
    assert out["n_gpus"] == 1 and out["scaling"] == "strong"
    assert out["config"]["backend"] == "nccl" and out["config"]["collectives_per_step"] == 1
    assert abs(out["value"] - 512 / (out["ms_per_step"] / 1e3)) <= 1e-6 * out["value"]
