"""GPU: the InnerState-compatible primitives (Sparse.py mirror) through pfr_solve / pfr_matvec."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from plate_inverse_problem_amd import Sparse

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _random_system(n=40, density=0.15, seed=0, batch=5):
    rng = np.random.default_rng(seed)
    A = sp.random(n, n, density=density, random_state=seed, format="coo")
    A = (A + A.T + sp.eye(n) * n).tocoo()              # structurally symmetric, diagonally dominant
    idx = np.stack([A.row, A.col], axis=1)
    (rows, cols), num = Sparse.create_symbolic(n, idx, np.complex128)
    base = np.asarray(A.tocsr()[rows, cols]).ravel()
    data = base[None, :] * (1 + 0.3 * rng.standard_normal((batch, rows.size))) \
        + 0.1j * rng.standard_normal((batch, rows.size))
    b = rng.standard_normal((batch, n)) + 1j * rng.standard_normal((batch, n))
    return n, rows, cols, num, data, b


def _dense(n, rows, cols, d):
    M = np.zeros((n, n), dtype=complex)
    M[rows, cols] = d
    return M


@pytest.mark.parametrize("transpose", [False, True])
def test_spsolve_batched_matches_dense(transpose):
    n, rows, cols, num, data, b = _random_system()
    x = Sparse.spsolve(torch.tensor(data, device=DEV), torch.tensor(b, device=DEV), solver_num=num,
                       transpose=transpose, n_cpu=0).cpu().numpy()
    for q in range(data.shape[0]):
        M = _dense(n, rows, cols, data[q])
        xd = np.linalg.solve(M.T if transpose else M, b[q])
        assert np.linalg.norm(x[q] - xd) / np.linalg.norm(xd) < 1e-12


def test_spsolve_broadcast_modes():
    n, rows, cols, num, data, b = _random_system(batch=3)
    d0 = torch.tensor(data[0], device=DEV)
    x1 = Sparse.spsolve(d0, torch.tensor(b, device=DEV), solver_num=num).cpu().numpy()        # mode 2
    x2 = Sparse.spsolve(torch.tensor(data, device=DEV), torch.tensor(b[0], device=DEV), solver_num=num)  # mode 1
    M0 = _dense(n, rows, cols, data[0])
    assert np.allclose(x1, np.linalg.solve(M0, b.T).T, rtol=1e-11)
    for q in range(3):
        assert np.allclose(x2[q].cpu().numpy(), np.linalg.solve(_dense(n, rows, cols, data[q]), b[0]), rtol=1e-11)
    x3 = Sparse.spsolve(torch.tensor(data, device=DEV), torch.tensor(np.stack([b, 2 * b]), device=DEV),
                        solver_num=num)                                                      # mode 4
    assert x3.shape == (2, 3, n) and torch.allclose(x3[1], 2 * x3[0])


@pytest.mark.parametrize("transpose", [False, True])
def test_mode4_multi_rhs_matches_dense(transpose):
    """Mode 4 (b (J, B, N), jax.hessian's batching): J right-hand sides per matrix on one
    factorisation (pfr_solve_multi); also with one broadcast matrix and across chunks."""
    n, rows, cols, num, data, b = _random_system(batch=5)
    rng = np.random.default_rng(3)
    bj = np.stack([b, rng.standard_normal(b.shape) + 1j * rng.standard_normal(b.shape), 3 * b])
    x = Sparse.spsolve(torch.tensor(data, device=DEV), torch.tensor(bj, device=DEV), solver_num=num,
                       transpose=transpose).cpu().numpy()
    assert x.shape == bj.shape
    for q in range(5):
        M = _dense(n, rows, cols, data[q])
        M = M.T if transpose else M
        for j in range(3):
            xd = np.linalg.solve(M, bj[j, q])
            assert np.linalg.norm(x[j, q] - xd) / np.linalg.norm(xd) < 1e-12
    xb = Sparse.spsolve(torch.tensor(data[0], device=DEV), torch.tensor(bj, device=DEV), solver_num=num)
    M0 = _dense(n, rows, cols, data[0])
    assert np.allclose(xb.cpu().numpy()[1, 2], np.linalg.solve(M0, bj[1, 2]), rtol=1e-11)


def test_mode4_gradcheck():
    n, rows, cols, num, data, b = _random_system(n=12, density=0.3, batch=2)
    d = torch.tensor(data, device=DEV, requires_grad=True)
    bj = torch.tensor(np.stack([b, 1j * b[::-1]]), device=DEV, requires_grad=True)
    fn = lambda d_, b_: Sparse.spsolve(d_, b_, solver_num=num)          # noqa: E731
    assert torch.autograd.gradcheck(fn, (d, bj), eps=1e-7, atol=1e-6, rtol=1e-5)


@pytest.mark.parametrize("transpose", [False, True])
def test_matvec(transpose):
    n, rows, cols, num, data, b = _random_system()
    y = Sparse.matvec(torch.tensor(data, device=DEV), torch.tensor(b, device=DEV), solver_num=num,
                      transpose=transpose).cpu().numpy()
    for q in range(data.shape[0]):
        M = _dense(n, rows, cols, data[q])
        assert np.allclose(y[q], (M.T if transpose else M) @ b[q], rtol=1e-12)


def test_spsolve_gradcheck():
    n, rows, cols, num, data, b = _random_system(n=12, density=0.3, batch=2)
    d = torch.tensor(data, device=DEV, requires_grad=True)
    bb = torch.tensor(b, device=DEV, requires_grad=True)
    fn = lambda d_, b_: Sparse.spsolve(d_, b_, solver_num=num)          # noqa: E731
    assert torch.autograd.gradcheck(fn, (d, bb), eps=1e-7, atol=1e-6, rtol=1e-5)
    fnt = lambda d_, b_: Sparse.matvec(d_, b_, solver_num=num, transpose=True)   # noqa: E731
    assert torch.autograd.gradcheck(fnt, (d, bb), eps=1e-7, atol=1e-6, rtol=1e-5)


def test_real_dtype_and_errors():
    n, rows, cols, num, data, b = _random_system(batch=2)
    xr = Sparse.spsolve(torch.tensor(data.real, device=DEV), torch.tensor(b.real, device=DEV), solver_num=num)
    assert xr.dtype == torch.float64
    M = _dense(n, rows, cols, data[1].real).real
    assert np.allclose(xr[1].cpu().numpy(), np.linalg.solve(M, b[1].real), rtol=1e-11)
    with pytest.raises(ValueError):
        Sparse.spsolve(torch.tensor(data, device=DEV), torch.tensor(b.real, device=DEV), solver_num=num)
    with pytest.raises(TypeError):
        Sparse.spsolve(torch.tensor(data, device=DEV), torch.tensor(b, device=DEV), solver_num=1.0)
