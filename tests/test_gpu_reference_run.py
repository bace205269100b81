"""GPU: the HIP path against outputs of the REFERENCE's own code (tests/golden/reference_run.npz,
see tests/test_reference_run.py), the optimisers' trajectories, and the exact Hessian against the
oracle.

Tolerances (ny = 3, fp64): fr <= 2e-9, losses <= 1e-8 relative (roundoff of the assembly order),
scaled gradient <= 1e-6 against central differences of the reference loss; optimiser iterates
<= 1e-7 (x) and 1e-6 (f); Hessian <= 1e-5 against central differences of the oracle's adjoint
gradient (the reference forms it as jax.jacobian(jax.grad(f)), Optimizers.py:125-136).
"""
import os

import numpy as np
import pytest
import torch

from helpers import make_problem, oracle_for

pytestmark = pytest.mark.gpu

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_run.npz"))
FREQS = G["freqs"]
MATS = ("isotropic", "orthotropic", "orthotropic_d4", "sol")
LOSSES = ("MSE", "RMSE", "MSE_AFC", "MSE_LOG_AFC")


@pytest.mark.parametrize("material", MATS)
def test_gpu_matches_reference_code(material):
    p = make_problem(material, ny=3, device="cuda:0")
    th0, th, ref = G[f"{material}_theta0"], G[f"{material}_theta"], G[f"{material}_ref"]
    fr = p.solveForward(FREQS, th0)
    assert np.max(np.abs(fr / G[f"{material}_fr"] - 1)) < 2e-9
    for lt in LOSSES:
        val = p.getLossFunction(FREQS, ref, lt)(torch.tensor(th)).item()
        assert abs(val / G[f"{material}_{lt}_loss"] - 1) < 1e-8, lt
    x = torch.tensor(th / th0, requires_grad=True)
    p.getLossFunction(FREQS, ref, "MSE_LOG_AFC", th0)(x).backward()
    g_ref = G[f"{material}_MSE_LOG_AFC_grad_scaled"]
    assert np.max(np.abs(x.grad.numpy() - g_ref)) / np.max(np.abs(g_ref)) < 1e-6


@pytest.mark.parametrize("opt", ["gd", "cd"])
def test_gpu_optimiser_trajectory_matches_reference(opt):
    from plate_inverse_problem_amd import Optimizers
    p = make_problem("orthotropic", ny=3, device="cuda:0")
    th0, th = G["orthotropic_theta0"], G["orthotropic_theta"]
    f = p.getLossFunction(FREQS, G["orthotropic_ref"], "MSE_LOG_AFC", th0)
    fn = Optimizers.optimize_gd if opt == "gd" else Optimizers.optimize_cd
    res = fn(f, th / th0, N_steps=3, h=0.05)
    xs = np.array([np.asarray(v, dtype=np.float64) for v in res.x_history + [res.x]])
    fs = np.array([float(v) for v in res.f_history + [res.f]])
    assert np.max(np.abs(xs - G[f"orthotropic_{opt}_x"])) < 1e-7
    assert np.max(np.abs(fs / G[f"orthotropic_{opt}_f"] - 1)) < 1e-6


def test_gpu_lbfgs_trajectory_matches_oracle_driven():
    """L-BFGS (this build's C5 driver; the reference has none) driven by the GPU loss + gradient and
    by the oracle's loss + adjoint gradient: the same iterates."""
    from oracle_loss import oracle_loss_fn
    from plate_inverse_problem_amd import Optimizers
    p = make_problem("orthotropic", ny=3, device="cuda:0")
    th0, th, ref = G["orthotropic_theta0"], G["orthotropic_theta"], G["orthotropic_ref"]
    runs = []
    for f in (p.getLossFunction(FREQS, ref, "MSE_LOG_AFC", th0),
              oracle_loss_fn(oracle_for(p), FREQS, ref, "MSE_LOG_AFC", scaling=th0)):
        res = Optimizers.optimize_lbfgs(f, th / th0, N_steps=3)
        runs.append((np.array([np.asarray(v, dtype=np.float64) for v in res.x_history + [res.x]]),
                     np.array([float(v) for v in res.f_history + [res.f]])))
    (xg, fg), (xo, fo) = runs
    assert xg.shape == xo.shape and len(xg) >= 3
    assert np.max(np.abs(xg - xo)) < 1e-7
    assert np.max(np.abs(fg / fo - 1)) < 1e-6


@pytest.mark.parametrize("material,loss_type", [("orthotropic", "MSE_LOG_AFC"), ("isotropic", "RMSE")])
def test_gpu_hessian_matches_oracle_differences(material, loss_type):
    from oracle.plate_oracle import loss_and_grad
    p = make_problem(material, ny=3, device="cuda:0")
    th0, ref = G[f"{material}_theta0"], G[f"{material}_ref"]
    x = G[f"{material}_theta"] / th0
    f, g, H = p.getLossHessianFunction(FREQS, ref, loss_type, th0)(x)
    orc = oracle_for(p)
    n = x.size
    Hfd = np.zeros((n, n))
    for j in range(n):
        h = 1e-4 * abs(x[j])
        gs = []
        for m in (-2, -1, 1, 2):
            t = x.copy()
            t[j] += m * h
            gs.append(loss_and_grad(orc, FREQS, ref, loss_type, t, scaling=th0)[1])
        Hfd[:, j] = (gs[0] - 8 * gs[1] + 8 * gs[2] - gs[3]) / (12 * h)
    Hfd = 0.5 * (Hfd + Hfd.T)
    lo, go = loss_and_grad(orc, FREQS, ref, loss_type, x, scaling=th0)
    assert abs(f / lo - 1) < 1e-8
    assert np.max(np.abs(g - go)) / np.max(np.abs(go)) < 1e-7
    assert np.max(np.abs(H - Hfd)) / np.max(np.abs(Hfd)) < 1e-5
