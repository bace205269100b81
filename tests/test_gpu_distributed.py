"""GPU: the product's multi-rank path -- Problem.getLossFunction(distributed=True) and
solveInverse(..., distributed=True) -- with two ranks on cuda:0 (gloo process group, 127.0.0.1).

Each rank sweeps its contiguous block of the frequencies on the device; one all_reduce(SUM) of the
packed [loss_sum, w_0..w_17] partials per evaluation (distributed.all_reduce_sum) gives every rank
the full loss and gradient, and every rank runs the identical optimiser.  Loss, gradient and the
L-BFGS iterates must equal the single-process run's (summation order differs: relative 1e-12).
Both ranks use max_batch = 64 so that two processes' device workspaces stay small.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

FREQS = np.linspace(50.0, 550.0, 150)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(distributed):
    from helpers import make_problem
    p = make_problem("orthotropic", ny=4, device="cuda:0", max_batch=64)
    theta0 = np.asarray(p.parameters, dtype=np.float64)
    ref = p.solveForward(FREQS) * np.exp(0.05j) * 1.02
    loss = p.getLossFunction(FREQS, ref, "MSE_LOG_AFC", distributed=distributed)
    x = torch.tensor(theta0 * 1.04, requires_grad=True)
    v = loss(x)
    v.backward()
    res = p.solveInverse(np.full(theta0.size, 0.03), "MSE_LOG_AFC", "lbfgs", ref_fr=(FREQS, ref), use_rel=True,
                         use_scaling=True, report=False, log=False, distributed=distributed, N_steps=3)
    xs = np.array([np.asarray(t, dtype=np.float64) for t in res.x_history + [res.x]])
    return float(v.item()), x.grad.numpy().copy(), xs


def _worker(rank, world, port, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out_q.put((rank,) + _run(True))
    except Exception as e:          # report instead of hanging the parent
        out_q.put((rank, repr(e), None, None))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_two_ranks_on_one_gpu_match_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = sorted([q.get(timeout=240) for _ in procs], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
    for r in res:
        assert r[2] is not None, r[1]
    assert all(pr.exitcode == 0 for pr in procs)
    (_, v0, g0, x0), (_, v1, g1, x1) = res
    assert v0 == v1 and np.array_equal(g0, g1) and np.array_equal(x0, x1)    # identical on every rank
    v, g, xs = _run(False)
    assert abs(v0 / v - 1) < 1e-12
    assert np.max(np.abs(g0 - g)) <= 1e-12 * np.max(np.abs(g))
    assert x0.shape == xs.shape and np.max(np.abs(x0 - xs) / np.abs(xs)) < 1e-9
