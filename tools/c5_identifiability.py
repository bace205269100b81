"""C5 identifiability: the exact Hessian of the C5 loss at theta_true and what it says about the
parameters the L-BFGS fit leaves at their start values.

The reference's trust-region model uses ``jax.jacobian(jax.grad(f))`` (Optimizers.py:125-136); here
``Problem.getLossHessianFunction`` (factors reused, pfr_hessian_sweep) evaluates the same exact
second derivatives.  Coordinates: relative parameters p = theta / theta_true (solveInverse's
use_rel), so H is dimensionless and its eigenvectors compare parameters of different units.

At theta_true the loss is zero and stationary, so near it L(p) ~ 1/2 (p - 1)^T H (p - 1).  Given the
L-BFGS end point (tools/c5_lbfgs.py, run here), the script decomposes its error e = p_end - 1 on H's
eigenvectors and reports per eigen-direction the error component and its loss share 1/2 lambda c^2:
if the parameters left near their start values (E2, nu12, b2..b4 in round 2) span the eigenvectors
of the smallest eigenvalues -- the directions along which a ~1 % move changes the loss by less than
the fit's final loss -- the plateau is a property of the measurement (one accelerometer on a strip),
not of the solver or its gradient.

    python tools/c5_identifiability.py [--ny 25] [--freqs 4096] [--out profiles/r03/c5_identifiability.json]
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
sys.path.insert(0, os.path.join(REPO, "tests"))

NAMES = ["E1", "E2", "G12", "nu12", "b1", "b2", "b3", "b4"]
REL0 = np.array([0.02, -0.02, 0.03, 0.01, 0.05, -0.05, 0.04, 0.03])     # tools/c5_lbfgs.py start


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ny", type=int, default=25)
    ap.add_argument("--freqs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    from helpers import make_problem
    from plate_inverse_problem_amd import Optimizers
    p = make_problem("orthotropic_d4", ny=a.ny, device="cuda:0")
    th = np.asarray(p.parameters, dtype=np.float64)
    freqs = np.linspace(40.0, 600.0, a.freqs)
    ref = p.solveForward(freqs)
    # exact Hessian at theta_true in relative coordinates
    t0 = time.perf_counter()
    model = p.getLossHessianFunction(freqs, ref, "MSE_LOG_AFC", scaling_params=th)
    f_true, g_true, H = model(np.ones(8))
    t_h = time.perf_counter() - t0
    lam, V = np.linalg.eigh(H)
    # the C5 fit from the perturbed start (same as tools/c5_lbfgs.py, one GPU)
    th0 = th * (1 + REL0)
    loss = p.getLossFunction(freqs, ref, "MSE_LOG_AFC", th0)
    res = Optimizers.optimize_lbfgs(loss, np.ones(8), N_steps=a.steps)
    p_end = np.asarray(res.x) * th0 / th                  # relative to theta_true
    e = p_end - 1.0
    c = V.T @ e
    share = 0.5 * lam * c ** 2
    # loss change of a 1 % move along each eigenvector, against the fit's final loss
    one_pct = 0.5 * lam * 1e-4
    out = {
        "workload": f"C5: orthotropic_d4, {p.mat_size} DOF x {a.freqs} freqs (40-600 Hz), MSE_LOG_AFC, "
                    "synthetic measurement at theta_true",
        "coordinates": "p = theta / theta_true (dimensionless); parameters " + ", ".join(NAMES),
        "hessian_s": t_h, "loss_at_true": f_true, "grad_at_true_maxabs": float(np.max(np.abs(g_true))),
        "hessian": H.tolist(), "eigenvalues": lam.tolist(),
        "eigenvectors": V.T.tolist(),
        "eigenvector_dominant_params": [[NAMES[j] for j in np.argsort(-np.abs(v))[:3]] for v in V.T],
        "condition_number": float(lam[-1] / max(lam[0], 1e-300)),
        "loss_of_1pct_move_along_eigvec": one_pct.tolist(),
        "fit": {"start_rel_error": REL0.tolist(), "end_rel_error": e.tolist(), "f_start": float(res.f_history[0]),
                "f_end": float(res.f), "iterations": int(res.niter) + 1, "status": res.status},
        "end_error_on_eigvecs": c.tolist(),
        "loss_share_per_eigvec": share.tolist(),
        "quadratic_model_loss": float(0.5 * e @ H @ e),
    }
    print(json.dumps({k: v for k, v in out.items() if k not in ("hessian", "eigenvectors")}, indent=1), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
