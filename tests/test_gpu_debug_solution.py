"""GPU: ``pfr_debug_solution`` (the diagnostic accessor of include/pfr.h) returns the last chunk's forward
solution and fr adjoint in caller numbering -- checked against the oracle's matrices: A x = b to the
static-pivot solve's backward error, A^T mu = d fr / d x to the bottom-up passes' seed rounding, and fr(x)
against the oracle's fr.  (The round-4 gradient analysis, DESIGN.md section 4, read the GPU's vectors
through it.)"""
import numpy as np
import pytest
import torch

from helpers import make_problem, oracle_for

pytestmark = pytest.mark.gpu


def test_debug_solution_vectors_solve_the_oracle_system():
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    p = make_problem("orthotropic", ny=6, device="cuda:0")
    orc = oracle_for(p)
    freqs = np.linspace(40.0, 600.0, 100)
    theta = p.parameters * 1.03
    ref = orc.fr(freqs, p.parameters).astype(np.complex128)
    eng = p.engine(freqs.size)
    eng.set_coefficients(_coeffs18(p._transform(), torch.as_tensor(theta)).detach().numpy())
    dev = eng.device
    w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
    loss = torch.zeros(1, dtype=torch.float64, device=dev)
    eng.sweep(torch.as_tensor(freqs, device=dev), _native.LOSS_MSE_LOG_AFC,
              ref=torch.view_as_real(torch.as_tensor(ref, device=dev)), scale=1.0, loss=loss, w=torch.view_as_real(w))
    torch.cuda.synchronize()
    assert eng.n_lanes == 1
    sv = eng.solvers[0]
    c = orc.coefficients(theta)
    aU, aV, aW = orc.averaging_vectors()
    ts2 = orc.acc_ts ** 2
    fr_o = orc.fr(freqs, theta)
    for q in (0, 37, 99):
        f = freqs[q]
        A = orc.matrix(f, c).tocsc()
        b = orc.rhs_vec * orc.rhs_scale(f, c)
        x = sv.debug_solution(0, q)
        mu = sv.debug_solution(1, q)
        # componentwise backward errors (UMFPACK's omega1) of both solves
        r = b - A @ x
        den = abs(A) @ np.abs(x) + np.abs(b)
        assert np.max(np.abs(r)[den > 0] / den[den > 0]) < 1e-12, q
        U, V, W = aU @ x, aV @ x, aW @ x
        fr = np.sqrt(ts2 * abs(U) ** 2 + ts2 * abs(V) ** 2 + abs(W) ** 2)
        assert abs(fr / fr_o[q] - 1) < 5e-9, (q, fr, fr_o[q])
        g = (ts2 * np.conj(U) * aU + ts2 * np.conj(V) * aV + np.conj(W) * aW) / fr
        ra = g - A.T @ mu
        dena = abs(A.T) @ np.abs(mu) + np.abs(g)
        # mu was solved for the seed of the bottom-up passes' fr (PFR_FN_DOT), which differs from the seed of x
        # by the solve's own rounding: its backward error against g(x) is that difference, not ~1e-15
        assert np.max(np.abs(ra)[dena > 0] / dena[dena > 0]) < 1e-8, q
    with pytest.raises(_native.NativeError):
        sv.debug_solution(2, 0)
