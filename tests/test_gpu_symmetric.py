"""GPU: symmetric mode (pfr_symbolic_options.symmetric) against the general LU path and the oracle.

Every FE matrix of the reference model is complex symmetric once the Dirichlet rows (only a
diagonal entry, tgv = -1, pyFFInterface.py:176) and their columns are taken out, so the
engine factorises A = L diag(U) L^T-style (U never formed, Dirichlet columns moved to the
right-hand side / the adjoint's Dirichlet rows).  Both paths must meet
the parity tolerances of test_gpu_parity.py; PFR_SYMMETRIC=0 selects the general path.
"""
import numpy as np
import pytest
import torch

from helpers import make_problem, oracle_for, report

pytestmark = pytest.mark.gpu

# as test_gpu_parity.py (the ny <= 6 conditioning band); measured round 2: fr <= 1.3e-9, loss
# <= 2.1e-9, gradient <= 9.8e-9 (general mode, ny = 5)
FR_RTOL = 5e-9
GRAD_RTOL = 1e-7


def _rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(np.max(np.abs(b)), 1e-300))


@pytest.mark.parametrize("material", ["isotropic", "orthotropic", "orthotropic_d4", "sol", "sol_sym", "symm_sol"])
def test_symmetric_mode_selected(material):
    p = make_problem(material, ny=3, device="cuda:0")
    eng = p.engine()
    assert eng.symmetric
    st = eng.sym.stats()
    assert st["symmetric"] == 1 and st["n_dirichlet"] > 0


@pytest.mark.parametrize("mode", ["symmetric", "general"])
@pytest.mark.parametrize("material,loss_type", [("orthotropic", "MSE_LOG_AFC"), ("sol", "MSE_AFC")])
def test_both_modes_match_oracle(mode, material, loss_type, monkeypatch):
    from oracle.plate_oracle import loss_and_grad
    monkeypatch.setenv("PFR_SYMMETRIC", "1" if mode == "symmetric" else "0")
    p = make_problem(material, ny=5, device="cuda:0")
    assert p.engine().symmetric == (mode == "symmetric")
    freqs = np.linspace(40.0, 600.0, 90)
    orc = oracle_for(p)
    fr = p.solveForward(freqs)
    assert _rel(fr, orc.fr(freqs, p.parameters)) < FR_RTOL
    ref = fr * np.exp(0.1j) * 1.02
    theta = p.parameters * 1.04
    x = torch.tensor(theta, requires_grad=True)
    val = p.getLossFunction(freqs, ref, loss_type)(x)
    val.backward()
    lo, go = loss_and_grad(orc, freqs, ref, loss_type, theta)
    report(f"modes {mode} {material}", fr_rel=_rel(fr, orc.fr(freqs, p.parameters)),
           loss_rel=abs(val.item() - lo) / abs(lo), grad_rel=_rel(x.grad.numpy(), go))
    assert abs(val.item() - lo) / abs(lo) < FR_RTOL
    assert _rel(x.grad.numpy(), go) < GRAD_RTOL


def test_general_mode_at_c2_size(monkeypatch):
    """General (non-symmetric) LU at the C2 size (isotropic, ny = 12, fronts up to 80 rows):
    forward sweep against the extended-precision fixture, loss + gradient against the oracle."""
    import os
    from oracle.plate_oracle import loss_and_grad
    monkeypatch.setenv("PFR_SYMMETRIC", "0")
    T = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c2_truth.npz"))
    p = make_problem("isotropic", ny=12, device="cuda:0")
    assert not p.engine().symmetric
    freqs = np.linspace(40.0, 600.0, 1024)
    fr = p.solveForward(freqs)
    idx = T["index"]
    e_fr = _rel(fr[idx] / T["fr_true"], np.ones(idx.size))
    f = freqs[idx]
    ref = fr[idx] * np.exp(0.1j) * 1.02
    theta = p.parameters * np.array([1.03, 0.98, 1.1])
    x = torch.tensor(theta, requires_grad=True)
    val = p.getLossFunction(f, ref, "MSE_LOG_AFC")(x)
    val.backward()
    lo, go = loss_and_grad(oracle_for(p), f, ref, "MSE_LOG_AFC", theta)
    report("general mode C2", fr_vs_truth=e_fr, loss_rel=abs(val.item() - lo) / abs(lo),
           grad_rel=_rel(x.grad.numpy(), go))
    assert e_fr < 5e-7                                  # the C2 band (test_gpu_fullsize.py)
    assert abs(val.item() - lo) / abs(lo) < 5e-7
    assert _rel(x.grad.numpy(), go) < 5e-6


def test_general_mode_hessian_matches_symmetric(monkeypatch):
    """The exact Hessian (tangent and second-order adjoint solves with the Dirichlet
    corrections) agrees between the two factorisations."""
    freqs = np.linspace(40, 600, 96)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("PFR_SYMMETRIC", mode)
        p = make_problem("orthotropic", ny=4, device="cuda:0")
        ref = p.solveForward(freqs).astype(np.complex128)
        theta0 = np.asarray(p.parameters, dtype=np.float64)
        model = p.getLossHessianFunction(freqs, ref * 1.03, "MSE_LOG_AFC", theta0)
        out[mode] = model(np.array([1.03, 0.98, 1.04, 1.02, 1.05]))
    f1, g1, H1 = out["1"]
    f0, g0, H0 = out["0"]
    assert abs(f1 - f0) <= 1e-9 * abs(f0)
    assert _rel(g1, g0) < 1e-7
    assert _rel(H1, H0) < 1e-6


def test_explicit_solve_refused_on_symmetric_solver():
    from plate_inverse_problem_amd import _native
    p = make_problem("isotropic", ny=3, device="cuda:0")
    eng = p.engine()
    n, nnz = p.mat_size, eng.keep.size
    data = torch.zeros((1, nnz), dtype=torch.complex128, device="cuda:0")
    b = torch.zeros((1, n), dtype=torch.complex128, device="cuda:0")
    x = torch.zeros_like(b)
    with pytest.raises(_native.NativeError, match="general analysis"):
        eng.solver.solve(torch.view_as_real(data), nnz, torch.view_as_real(b), n, torch.view_as_real(x), False, 1)


@pytest.mark.parametrize("blk_min", ["0", "4", "24"])
def test_schur_kernel_split_matches_oracle(blk_min, monkeypatch):
    """Symmetric Schur complement through the 4 x 4 tile kernel alone (PFR_SCHUR_BLK_MIN=0),
    the LDS block kernel for almost every front (4) and the default split (24)."""
    monkeypatch.setenv("PFR_SCHUR_BLK_MIN", blk_min)
    p = make_problem("orthotropic", ny=6, device="cuda:0")
    freqs = np.linspace(40.0, 600.0, 130)
    fr = p.solveForward(freqs)
    report(f"schur split {blk_min}", fr_rel=_rel(fr, oracle_for(p).fr(freqs, p.parameters)))
    assert _rel(fr, oracle_for(p).fr(freqs, p.parameters)) < FR_RTOL
