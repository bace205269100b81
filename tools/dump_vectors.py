"""Diagnostic: the GPU's forward solutions and adjoints of one 64-frequency group of the C3 sweep, for a
CPU-side comparison with the extended-precision solutions (tools/compare_vectors.py).

    python tools/dump_vectors.py --out gpurun_out/vec.npz [--group 19] [--lanes 28:52] [--modes 11,27]

One loss + gradient sweep per check mode over the group's 64 frequencies (engine sized for the full
4,096-frequency sweep, as the bench); x and the adjoint of the listed lanes through pfr_debug_solution,
plus the group's unscaled partial sums.
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--group", type=int, default=19)
    ap.add_argument("--lanes", default="28:52")
    ap.add_argument("--modes", default="11,27")
    args = ap.parse_args()
    from helpers import make_problem
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    T = np.load(os.path.join(REPO, "tests", "golden", "c3_grad_truth.npz"))
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    theta = np.asarray(T["theta"])
    eng = p.engine(4096)
    eng.set_coefficients(_coeffs18(p._transform(), torch.as_tensor(theta)).detach().numpy())
    dev = eng.device
    sel = np.arange(args.group * 64, args.group * 64 + 64)
    a, b = (int(v) for v in args.lanes.split(":"))
    out = {"index": sel[a:b], "lanes": np.arange(a, b)}
    for mode in (int(m) for m in args.modes.split(",")):
        eng.set_check(mode)
        f = torch.as_tensor(T["freqs"][sel], device=dev)
        ref = torch.as_tensor(T["ref"][sel].astype(np.complex128), device=dev)
        w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        eng.sweep(f, _native.LOSS_MSE_LOG_AFC, ref=torch.view_as_real(ref), scale=1.0, loss=loss,
                  w=torch.view_as_real(w))
        torch.cuda.synchronize()
        out[f"w_{mode}"] = eng.expand(w).cpu().numpy()
        out[f"x_{mode}"] = np.stack([eng.solvers[0].debug_solution(0, q) for q in range(a, b)])
        out[f"mu_{mode}"] = np.stack([eng.solvers[0].debug_solution(1, q) for q in range(a, b)])
        wt = T["w_true"][sel].sum(0)
        print(f"mode {mode}: group err {np.max(np.abs(out[f'w_{mode}'] - wt)) / np.max(np.abs(T['w_true'].sum(0))):.2e}",
              flush=True)
    np.savez(args.out, **out)


if __name__ == "__main__":
    main()
