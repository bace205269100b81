"""Local optimisers over the differentiable loss (``source/jax_plate/Optimizers.py``).

Same names, arguments and ``optResult`` as the reference; ``jax.value_and_grad``
becomes one fused forward + adjoint GPU sweep (``Problem.getLossFunction``).
Additions: ``optimize_lbfgs`` (two-loop L-BFGS with a capped step and Armijo
backtracking, the BASELINE.json C5 driver).  The trust-region Newton model
(``Optimizers.py:125-136``, JAX forward-over-reverse there) takes the EXACT Hessian
from ``Problem.getLossHessianFunction`` when ``solveInverse`` passes it as ``model``
(one factorisation + forward/adjoint/second-order solves per evaluation, factors
reused on the device; ``solveInverse(..., exact_hessian=False)`` opts out); called
without ``model`` it falls back to central differences of the adjoint gradient
(2 n_theta extra fused sweeps).
"""
from __future__ import annotations

from collections import namedtuple
from typing import Callable

import numpy as np
import torch

optResult = namedtuple("optResult", ["x", "f", "f_history", "x_history", "grad_history", "niter", "status"])


def _t(x) -> torch.Tensor:
    return torch.as_tensor(np.asarray(x, dtype=np.float64) if not isinstance(x, torch.Tensor) else x,
                           dtype=torch.float64).detach().cpu()


def value_and_grad(f: Callable) -> Callable:
    """``x -> (f(x), df/dx)`` as numpy (one fused forward + adjoint sweep)."""
    def vg(x):
        xt = _t(x).clone().requires_grad_(True)
        val = f(xt)
        (g,) = torch.autograd.grad(val, xt)
        return float(val.detach()), g.numpy().copy()
    return vg


def fd_hessian(grad: Callable, x: np.ndarray, rel: float = 1e-4) -> np.ndarray:
    """Symmetrised central-difference Jacobian of the gradient."""
    n = x.size
    H = np.zeros((n, n))
    for j in range(n):
        h = rel * abs(x[j]) if x[j] != 0 else rel
        e = np.zeros(n)
        e[j] = h
        H[:, j] = (grad(x + e) - grad(x - e)) / (2 * h)
    return 0.5 * (H + H.T)


def _sd_and_norm(B, g, lam):
    sd = np.linalg.solve(B + lam * np.eye(B.shape[0]), -g)
    return sd, np.linalg.norm(sd)


def solve_trust_region_model(B, g, delta, rtol=1e-6, max_iter=100):
    """min g.p + p.B.p/2 s.t. |p| <= delta by bisection on the shift (Optimizers.py:69-122)."""
    lams = np.linalg.eigvalsh(B)
    sd = np.linalg.solve(B, -g)
    if np.linalg.norm(sd) <= delta and lams.min() >= 0:
        return sd, 0.0, -(g @ sd + 0.5 * sd @ B @ sd)
    l_left = max(0.0, (-lams).max())
    l_right = l_left + 1.0
    sd, pnorm = _sd_and_norm(B, g, l_right)
    for _ in range(max_iter):
        if pnorm <= delta:
            break
        l_left, l_right = l_right, 2.0 * l_right
        sd, pnorm = _sd_and_norm(B, g, l_right)
    if pnorm > delta:
        raise AssertionError("Failed to find upper bound for lambda")
    lam = l_right
    for _ in range(2 * max_iter):
        if pnorm <= delta and delta - pnorm <= delta * rtol:
            break
        lam = 0.5 * (l_right + l_left)
        sd, pnorm = _sd_and_norm(B, g, lam)
        if pnorm < delta:
            l_right = lam
        else:
            l_left = lam
    if pnorm > delta:
        lam = l_right
        sd, pnorm = _sd_and_norm(B, g, lam)
    pred = -(g @ sd + 0.5 * sd @ B @ sd)
    if pred < 0:
        raise AssertionError("Predicted improvement for quadratic model is negative")
    return sd, lam, pred


def optimize_trust_region(f, x_0, N_steps=10, delta_max=1.0, delta=None, eta=0.15, method="newt",
                          steps_to_stall=10, hessian_rel_step=1e-4, model=None):
    """Trust-region Newton (``Optimizers.py:147-232`` of the reference).  ``model(x) -> (f, g, H)``
    supplies the exact Hessian (``Problem.getLossHessianFunction``: factors reused on the GPU);
    without it the Hessian is central differences of the adjoint gradient."""
    if delta is None:
        delta = delta_max / 10.0
    if not 0 <= eta <= 0.25:
        raise ValueError(f"eta should be in [0, 0.25]; got {eta:f}")
    if method != "newt":
        raise NotImplementedError(f"Method <<{method}>> not implemented")
    vg = value_and_grad(f)
    grad = lambda x: vg(x)[1]                                   # noqa: E731
    x = np.asarray(x_0, dtype=np.float64).copy()
    f_hist, x_hist, g_hist = [], [], []
    status, stall, need_model = "Running", 0, True
    cur_f, g, B = None, None, None
    k = 0
    for k in range(N_steps):
        if need_model:
            if model is not None:
                cur_f, g, B = model(x)
            else:
                cur_f, g = vg(x)
                B = fd_hessian(grad, x, hessian_rel_step)
        try:
            sd, lam, pred = solve_trust_region_model(B, g, delta)
        except AssertionError as e:
            status = str(e)
            break
        new_f = float(f(_t(x + sd)))
        rho = (cur_f - new_f) / pred if pred > 0 else -np.inf
        if rho < 0.25:
            delta /= 4.0
        elif rho >= 0.75 and lam > 0.0:
            delta = min(2.0 * delta, delta_max)
        if rho >= eta:
            x = x + sd
            need_model, stall = True, 0
        else:
            need_model, stall = False, stall + 1
        f_hist.append(cur_f)
        x_hist.append(x.copy())
        g_hist.append(g.copy())
        if cur_f < 1e-16:
            status = "Converged"
            break
        if stall >= steps_to_stall:
            status = "Stalled"
            break
    return optResult(x, cur_f, f_hist, x_hist, g_hist, k, status)


def optimize_gd(f, x_0, N_steps=100, h=0.01, f_min=1e-8):
    """Plain gradient descent x -= h g (Optimizers.py:231-254)."""
    vg = value_and_grad(f)
    x = np.asarray(x_0, dtype=np.float64).copy()
    f_hist, x_hist, g_hist = [], [], []
    status, cur_f, k = "Running", None, 0
    for k in range(N_steps):
        cur_f, g = vg(x)
        x_hist.append(x.copy())
        f_hist.append(cur_f)
        g_hist.append(g)
        if cur_f <= f_min:
            status = "Converged"
            break
        x = x - h * g
    return optResult(x, cur_f, f_hist, x_hist, g_hist, k, status)


def optimize_cd(f, x_0, N_steps=100, h=0.01, f_min=1e-8):
    """Coordinate descent, one coordinate per gradient evaluation (Optimizers.py:257-287)."""
    vg = value_and_grad(f)
    x = np.asarray(x_0, dtype=np.float64).copy()
    n = x.size
    assert n >= 2
    f_hist, x_hist, g_hist = [], [], []
    status, cur_f, k = "Running", None, 0
    for k in range(N_steps):
        for i in range(n):
            cur_f, g = vg(x)
            g = g * np.eye(n)[i]
            x_hist.append(x.copy())
            f_hist.append(cur_f)
            g_hist.append(g)
            if cur_f <= f_min:
                status = "Converged"
                break
            x = x - h * g
    return optResult(x, cur_f, f_hist, x_hist, g_hist, k, status)


def optimize_cd_mem2(f, x_0, N_steps=100, h=0.01, f_min=1e-8):
    """Coordinate descent with per-coordinate step back-off (Optimizers.py:326-367)."""
    vg = value_and_grad(f)
    x = np.asarray(x_0, dtype=np.float64).copy()
    n = x.size
    assert n >= 2
    hs = np.full(n, h, dtype=np.float64)
    f_hist, x_hist, g_hist = [], [], []
    status, cur_f, k = "Running", None, 0
    for k in range(N_steps):
        for i in range(n):
            cur_f, g = vg(x)
            g = g * np.eye(n)[i]
            x_hist.append(x.copy())
            f_hist.append(cur_f)
            g_hist.append(g)
            if cur_f <= f_min:
                status = "Converged"
                break
            x = x - hs[i] * g
            if float(f(_t(x))) > f_hist[-1]:
                hs[i] /= 5
                x = x_hist[-1] - hs[i] * g
    return optResult(x, cur_f, f_hist, x_hist, g_hist, k, status)


optimize_cd_mem = optimize_cd_mem2


def optimize_lbfgs(f, x_0, N_steps=50, history_size=10, max_step=0.05, c1=1e-4, max_backtrack=30,
                   tolerance_grad=1e-12, f_min=1e-16, rtol_f=1e-8):
    """L-BFGS (two-loop recursion) with Armijo backtracking.

    One fused forward + adjoint sweep per function evaluation.  Every trial step is
    capped at ``max_step`` (infinity norm, in the optimiser's coordinates): the FR
    misfit's basin in the stiffness moduli is only a few percent wide (resonances
    move past each other), so an unscaled gradient step -- or a quasi-Newton step
    whose curvature pair s.y is barely positive -- would leave it (and the loss far
    outside, with every resonance pushed past the band, can be LOWER than inside).
    """
    vg = value_and_grad(f)
    x = np.asarray(x_0, dtype=np.float64).copy()
    cur_f, g = vg(x)
    S, Y = [], []
    f_hist, x_hist, g_hist = [], [], []
    status, k = "Running", 0
    for k in range(N_steps):
        f_hist.append(cur_f)
        x_hist.append(x.copy())
        g_hist.append(g.copy())
        if cur_f <= f_min:
            status = "Converged"
            break
        if np.max(np.abs(g)) <= tolerance_grad:
            status = "Converged (gradient)"
            break
        q = -g.copy()
        alphas = []
        for s_, y_ in zip(reversed(S), reversed(Y)):
            a = (s_ @ q) / (y_ @ s_)
            alphas.append(a)
            q -= a * y_
        if S:
            q *= (S[-1] @ Y[-1]) / (Y[-1] @ Y[-1])
        for (s_, y_), a in zip(zip(S, Y), reversed(alphas)):
            q += (a - (y_ @ q) / (y_ @ s_)) * s_
        d = q
        gtd = g @ d
        if gtd >= 0:                                  # not a descent direction: restart
            S.clear()
            Y.clear()
            d = -g
            gtd = g @ d
        t = min(1.0, max_step / max(np.max(np.abs(d)), 1e-300))
        for _ in range(max_backtrack):
            x_new = x + t * d
            f_new, g_new = vg(x_new)
            if np.isfinite(f_new) and f_new <= cur_f + c1 * t * gtd:
                break
            t *= 0.5
        else:
            # no decrease along the capped direction: converged when the loss already sits at the
            # level of the fp64 sweep's rounding relative to where it started
            status = "Converged (no further decrease)" if cur_f <= rtol_f * f_hist[0] else "Line search failed"
            break
        s_, y_ = x_new - x, g_new - g
        if s_ @ y_ > 1e-300:
            S.append(s_)
            Y.append(y_)
            if len(S) > history_size:
                S.pop(0)
                Y.pop(0)
        x, cur_f, g = x_new, f_new, g_new
    return optResult(x, cur_f, f_hist, x_hist, g_hist, k, status)
