"""Worker of tests/test_gpu_nccl.py, run under ``torch.distributed.run`` (one rank per GPU).

Joins the process group the launcher describes (``distributed.init_from_env``: RCCL unless
PFR_DIST_BACKEND says otherwise), then drives the product's collective paths on device tensors:
``all_reduce_sum`` of a complex CUDA tensor, ``getLossFunction(..., distributed=True)`` (the
loss/gradient all-reduce) and ``solveForward(..., distributed=True)`` (the all-gather of fr),
each compared with the single-process result.  Rank 0 prints one JSON line.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    import plate_inverse_problem_amd.distributed as pdist
    import torch.distributed as dist
    rank, world, backend = pdist.init_from_env(device)
    assert backend is not None
    n0 = pdist.N_COLLECTIVES
    # 1. a complex device tensor through dist.all_reduce (summed over `world` ranks)
    t = torch.tensor([1.0 + 2.0j, -3.0 + 0.5j], dtype=torch.complex128, device=device) * (rank + 1)
    s = pdist.all_reduce_sum(t)
    expect = torch.tensor([1.0 + 2.0j, -3.0 + 0.5j], dtype=torch.complex128) * (world * (world + 1) / 2)
    assert s.device == device and torch.allclose(s.cpu(), expect)
    # 2. distributed loss + gradient against the single-process evaluation on this rank
    from helpers import make_problem
    p = make_problem("orthotropic", ny=4, device=device)
    freqs = np.linspace(60.0, 500.0, 96)
    ref = p.solveForward(freqs) * np.exp(0.05j) * 1.03
    theta = p.parameters * 1.05
    x = torch.tensor(theta, requires_grad=True)
    v = p.getLossFunction(freqs, ref, "MSE_LOG_AFC", distributed=True)(x)
    v.backward()
    y = torch.tensor(theta, requires_grad=True)
    v1 = p.getLossFunction(freqs, ref, "MSE_LOG_AFC")(y)
    v1.backward()
    loss_rel = abs(v.item() - v1.item()) / abs(v1.item())
    grad_rel = float((x.grad - y.grad).abs().max() / y.grad.abs().max())
    # 3. distributed solveForward (all-gather of the shards) against the full sweep
    fr_d = p.solveForward(freqs, distributed=True)
    fr_1 = p.solveForward(freqs)
    fr_rel = float(np.max(np.abs(fr_d - fr_1)) / np.max(np.abs(fr_1)))
    out = {"backend": backend, "world": world, "collectives": pdist.N_COLLECTIVES - n0, "loss_rel": loss_rel,
           "grad_rel": grad_rel, "fr_rel": fr_rel}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
