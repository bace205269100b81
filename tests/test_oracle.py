"""The oracle itself: dense cross-check, interpolation identity, adjoint vs FD,
physics sanity (clamped-free strip resonance)."""
import numpy as np
import pytest

from helpers import make_problem, oracle_for
from oracle import plate_oracle as orc


@pytest.fixture(scope="module")
def small():
    p = make_problem("orthotropic", ny=3)
    return p, oracle_for(p)


def test_sparse_lu_matches_dense(small):
    p, o = small
    c = o.coefficients(p.parameters)
    A = o.matrix(250.0, c)
    b = (o.rhs_vec * o.rhs_scale(250.0, c)).astype(complex)
    x = orc.sparse_lu(A).solve(b)
    xd = np.linalg.solve(A.toarray(), b)
    assert np.linalg.norm(x - xd) / np.linalg.norm(xd) < 1e-11
    xt = orc.sparse_lu(A).solve(b, trans="T")
    assert np.linalg.norm(xt - np.linalg.solve(A.toarray().T, b)) / np.linalg.norm(xt) < 1e-11


def test_dirichlet_rows_give_clamped_values(small):
    """Unit Dirichlet rows + rhs scale = diag: w = 1 on clamped vertices (pyFFInterface.py:185-197)."""
    p, o = small
    x, _, _ = o.solve(180.0, p.parameters)
    d = np.nonzero(p.vec)[0]
    assert np.allclose(x[d], 1.0, rtol=1e-12)


def test_averaging_vectors_equal_dense_interpolation(small):
    p, o = small
    x, _, _ = o.solve(200.0, p.parameters)
    U, V, W = o.uvw(x)
    aU, aV, aW = o.averaging_vectors()
    assert np.allclose([U, V, W], [aU @ x, aV @ x, aW @ x], rtol=1e-12)
    pa = p.averaging_vectors()
    assert all(np.allclose(a, b) for a, b in zip(pa, (aU, aV, aW)))


@pytest.mark.parametrize("loss_type", orc.LOSS_TYPES)
def test_adjoint_gradient_vs_finite_differences(small, loss_type):
    p, o = small
    freqs = np.linspace(60.0, 560.0, 9)
    ref = o.fr(freqs, p.parameters) * np.exp(0.2j)
    th = p.parameters * np.array([1.1, 0.95, 1.2, 1.05, 1.3])
    L, g = orc.loss_and_grad(o, freqs, ref, loss_type, th)
    gfd = orc.fd_grad(o, freqs, ref, loss_type, th)
    assert abs(L - orc.loss(o, freqs, ref, loss_type, th)) <= 1e-12 * abs(L)
    assert np.max(np.abs(g - gfd)) / np.max(np.abs(gfd)) < 1e-4     # FD truncation in the loss factor


def test_refactor_adjoint_mode_same_result(small):
    p, o = small
    freqs = np.linspace(100.0, 300.0, 4)
    ref = o.fr(freqs, p.parameters)
    th = p.parameters * 1.1
    a = orc.frequency_partials(o, freqs, ref, "MSE", th)
    b = orc.frequency_partials(o, freqs, ref, "MSE", th, refactor_adjoint=True)
    c = orc.frequency_partials(o, freqs, ref, "MSE", th, factorisations=3)    # the reference-faithful count
    assert np.isclose(a[0], b[0], rtol=1e-13) and np.allclose(a[1], b[1], rtol=1e-10)
    assert np.isclose(a[0], c[0], rtol=1e-13) and np.allclose(a[1], c[1], rtol=1e-10)


def test_first_resonance_near_euler_bernoulli():
    """Without accelerometer mass the steel strip's first bending mode is near
    f1 = (1.875^2 / 2 pi) sqrt(E h^2 / (12 rho)) / L^2 ~ 162 Hz (plate: +few %)."""
    p = make_problem("isotropic", ny=4)
    p.I0Corr = 0.0
    p.I2Corr = 0.0
    o = oracle_for(p)
    freqs = np.arange(140.0, 190.0, 1.0)
    fr = o.fr(freqs, p.parameters)
    f_peak = freqs[np.argmax(fr)]
    f_eb = 1.875 ** 2 / (2 * np.pi) * np.sqrt(200e9 * 2e-3 ** 2 / (12 * 7920.0)) / 0.1 ** 2
    assert abs(f_peak - f_eb) / f_eb < 0.06
    assert np.isclose(o.fr([1.0], p.parameters)[0], 1.0, atol=0.01)   # quasi-static: rigid base motion
