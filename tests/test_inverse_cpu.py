"""Host-side inverse-problem pieces on CPU: Compressor (pinned by the reference's
own class, tests/golden/compressor.npz) and the optimisers (driven by a torch
loss, the same callable protocol as getLossFunction)."""
import os

import numpy as np
import pytest
import torch

from plate_inverse_problem_amd import Optimizers as O
from plate_inverse_problem_amd.Input import Compressor

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "compressor.npz")


@pytest.mark.parametrize("alg", [0, 1])
@pytest.mark.parametrize("n", [100, 200, 300])
def test_compressor_matches_reference(alg, n):
    g = np.load(GOLDEN)
    fsel, frsel = Compressor(g["freqs"], g["fr"], 1500, alg)(n)
    assert np.array_equal(np.searchsorted(g["freqs"], fsel), g[f"alg{alg}_n{n}"])
    assert np.array_equal(frsel, g["fr"][g[f"alg{alg}_n{n}"]])


def test_compressor_rejects_oversize():
    g = np.load(GOLDEN)
    with pytest.raises(ValueError):
        Compressor(g["freqs"], g["fr"], 50, 0)(51)


def _quad():
    A = torch.tensor([[3.0, 0.5, 0.0], [0.5, 2.0, 0.3], [0.0, 0.3, 1.0]], dtype=torch.float64)
    xs = torch.tensor([1.0, -2.0, 0.5], dtype=torch.float64)
    return lambda x: 0.5 * (x - xs) @ A @ (x - xs), xs.numpy()


def test_gd_and_cd_decrease():
    f, xs = _quad()
    for fn in (O.optimize_gd, O.optimize_cd, O.optimize_cd_mem2):
        r = fn(f, np.zeros(3), N_steps=30, h=0.2)
        assert r.f < r.f_history[0] and len(r.x_history) == len(r.f_history)
        assert r.status in ("Running", "Converged")


def test_trust_region_converges():
    f, xs = _quad()
    r = O.optimize_trust_region(f, np.zeros(3), N_steps=30, delta_max=10.0)
    assert np.allclose(r.x, xs, atol=1e-5)


def test_trust_region_with_exact_model():
    """``model(x) -> (f, g, H)`` (Problem.getLossHessianFunction's contract) replaces the FD Hessian."""
    f, xs = _quad()
    A = np.array([[3.0, 0.5, 0.0], [0.5, 2.0, 0.3], [0.0, 0.3, 1.0]])
    calls = []

    def model(x):
        calls.append(x.copy())
        d = x - xs
        return 0.5 * d @ A @ d, A @ d, A

    r = O.optimize_trust_region(f, np.zeros(3), N_steps=30, delta_max=10.0, model=model)
    assert np.allclose(r.x, xs, atol=1e-10) and len(calls) >= 1


def test_lbfgs_converges():
    f, xs = _quad()
    r = O.optimize_lbfgs(f, np.zeros(3), N_steps=20, max_step=10.0)
    assert np.allclose(r.x, xs, atol=1e-7) and r.f < 1e-12


def test_trust_region_model_step_inside_radius():
    B = np.diag([2.0, -1.0])
    g = np.array([1.0, 1.0])
    sd, lam, pred = O.solve_trust_region_model(B, g, 0.5)
    assert np.linalg.norm(sd) <= 0.5 * (1 + 1e-6) and pred > 0 and lam > 1.0
