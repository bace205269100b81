"""The jet material transform (plate_inverse_problem_amd/_abd_jet.py) against the torch transforms of
Material.py: values to rounding and Jacobians against torch autograd, every material type; the custom
autograd Function's backward against autograd through the torch transform."""
import numpy as np
import pytest
import torch

from helpers import MATERIALS, make_problem
from plate_inverse_problem_amd._abd_jet import abd_and_jacobian, coeffs18
from plate_inverse_problem_amd.Problem import _coeffs18


@pytest.mark.parametrize("name", sorted(MATERIALS))
def test_jet_matches_torch_transform(name):
    p = make_problem(name, ny=2)
    h = p.geometry.height
    tr = p._transform()
    rng = np.random.default_rng(0)
    for trial in range(3):
        theta = p.parameters * (1 + 0.1 * rng.standard_normal(p.parameters.size))
        c, J = abd_and_jacobian(p.material, h, theta)
        ct = _coeffs18(tr, torch.as_tensor(theta)).numpy()
        scale = np.abs(ct).max()
        assert np.max(np.abs(c - ct)) <= 1e-14 * scale, name
        f = lambda x: torch.view_as_real(_coeffs18(tr, x)).reshape(-1)   # noqa: E731
        Jr = torch.autograd.functional.jacobian(f, torch.as_tensor(theta)).numpy()
        Jt = Jr[0::2] + 1j * Jr[1::2]
        for k in range(18):
            assert np.allclose(J[k], Jt[k], rtol=1e-12, atol=1e-14 * np.abs(Jt[k]).max() + 1e-300), (name, k)


@pytest.mark.parametrize("name", ["orthotropic", "orthotropic_d4", "sol"])
def test_jet_autograd_function_backward(name):
    p = make_problem(name, ny=2)
    tr = p._transform()
    theta = p.parameters * 1.07
    scaling = torch.as_tensor(np.linspace(0.5, 1.5, theta.size))
    g = torch.randn(18, dtype=torch.complex128, generator=torch.Generator().manual_seed(1))
    x1 = torch.tensor(theta, requires_grad=True)
    coeffs18(p.material, p.geometry.height, x1 * scaling).backward(g)
    x2 = torch.tensor(theta, requires_grad=True)
    _coeffs18(tr, x2 * scaling).backward(g)
    assert torch.allclose(x1.grad, x2.grad, rtol=1e-12, atol=0)
