"""C5 end to end on one GPU: L-BFGS over the 8 parameters of ``orthotropic_d4`` (4 moduli + 4 loss
factors) on the C3 mesh (ny = 25, 19,353 DOF) x 4,096 frequencies (BASELINE.json configs[4] on one
GPU; the 8-GPU run is the driver's).  Synthetic measurement: the forward sweep at theta_true;
start: theta_true * (1 + [0.02, -0.02, 0.03, 0.01, 0.05, -0.05, 0.04, 0.03]); loss MSE_LOG_AFC on
scaled parameters (solveInverse use_rel + use_scaling).

Prints one JSON line: iterations, loss history, relative parameter errors, wall time per
iteration and per loss + gradient evaluation.

    python tools/c5_lbfgs.py [--ny 25] [--freqs 4096] [--steps 30]

C5 proper (BASELINE.json configs[4]) is the same fit over N GPUs (C4's sharding: --freqs in total,
--weak for --freqs per GPU), one process per GPU:

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/c5_lbfgs.py

Each rank sweeps its contiguous block of the frequencies; one all-reduce of the loss and gradient
partials per evaluation (Problem.getLossFunction(..., distributed=True)); every rank runs the same
L-BFGS iterates, rank 0 prints.  PFR_BENCH_ONE_DEVICE=1 / PFR_DIST_BACKEND=gloo rehearse it on one
GPU (as bench.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ny", type=int, default=25)
    ap.add_argument("--freqs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--weak", action="store_true", help="--freqs per GPU instead of in total")
    a = ap.parse_args()
    import torch.distributed as dist
    local = 0 if os.environ.get("PFR_BENCH_ONE_DEVICE") == "1" else int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    from plate_inverse_problem_amd.distributed import init_from_env
    rank, world, backend = init_from_env(device)
    from plate_inverse_problem_amd.Accelerometer import Accelerometer
    from plate_inverse_problem_amd.Geometry import Geometry, GeometryParams
    from plate_inverse_problem_amd.Material import get_material
    from plate_inverse_problem_amd.Problem import Problem
    from plate_inverse_problem_amd import Optimizers

    acc = Accelerometer("AP1030")
    geom = Geometry("sh_i", acc, GeometryParams(100e-3, 20e-3, 2e-3, None, None), ny=a.ny)
    mat = get_material(1500.0, "orthotropic_d4", E1=120e9, E2=8e9, G12=5e9, nu12=0.3, b1=0.01, b2=0.02, b3=0.015,
                       b4=0.005)
    from plate_inverse_problem_amd.distributed import shard_range
    t0 = time.perf_counter()
    p = Problem(geom, mat, acc, device=device)
    n_total = a.freqs * world if a.weak else a.freqs
    freqs = np.linspace(40.0, 600.0, n_total)
    lo, hi = shard_range(n_total, rank, world)
    fr = np.zeros(n_total, dtype=np.complex128)
    fr[lo:hi] = p.solveForward(freqs[lo:hi])          # each rank measures its own block
    torch.cuda.synchronize()
    t_setup = time.perf_counter() - t0
    rel0 = np.array([0.02, -0.02, 0.03, 0.01, 0.05, -0.05, 0.04, 0.03])
    theta0 = np.asarray(p.parameters, dtype=np.float64)
    loss = p.getLossFunction(freqs, fr, "MSE_LOG_AFC", theta0 * (1 + rel0), distributed=backend is not None)
    n_eval = [0]

    def counted(x):
        n_eval[0] += 1
        return loss(x)

    t0 = time.perf_counter()
    res = Optimizers.optimize_lbfgs(counted, np.ones(8), N_steps=a.steps)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    x = np.asarray(res.x) * theta0 * (1 + rel0)
    if world > 1:
        t = torch.tensor([wall], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t.item())
    out = {"workload": f"C5 on {world} GPU(s): orthotropic_d4 L-BFGS, {p.mat_size} DOF x {n_total} freqs, MSE_LOG_AFC",
           "n_gpus": world, "n_dofs": p.mat_size, "freqs": n_total, "iterations": int(res.niter) + 1,
           "evaluations": n_eval[0],
           "status": res.status, "f_history": [float(v) for v in res.f_history] + [float(res.f)],
           "rel_error_start": rel0.tolist(), "rel_error_end": ((x - theta0) / theta0).tolist(),
           "wall_s": wall, "s_per_iteration": wall / (int(res.niter) + 1), "s_per_evaluation": wall / n_eval[0],
           "freq_solves_per_s": n_eval[0] * n_total / wall, "setup_s": t_setup}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if backend is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
