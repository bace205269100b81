"""GPU: per-frequency backward-error checks (pfr_set_check) and iterative refinement.

The reference's only failure detection is UMFPACK's status code (umfpack_interface.h:10-18), and
its solves refine by default (NULL Control at InnerState.h:246-247: UMFPACK_IRSTEP = 2).  A static
pivot order needs its own: after every solve the device computes the componentwise backward error
max_i |b - A x|_i / (|A||x| + |b|)_i and flags the frequencies above the tolerance.
"""
import numpy as np
import pytest
import torch

from helpers import make_problem, oracle_for

pytestmark = pytest.mark.gpu


def _general_solver(n, rows, cols, batch=64):
    from plate_inverse_problem_amd import _native
    order = np.lexsort((rows, cols))
    r, c = rows[order].astype(np.int32), cols[order].astype(np.int32)
    colptr = np.zeros(n + 1, np.int64)
    np.add.at(colptr, c.astype(np.int64) + 1, 1)
    sym = _native.Symbolic(n, np.cumsum(colptr).astype(np.int32), r)
    return _native.Solver(sym, 0, batch), r, c


def _pattern(n, rng):
    pairs = {(i, i) for i in range(n)} | {(i, i + 1) for i in range(n - 1)} | {(i + 1, i) for i in range(n - 1)}
    for _ in range(3 * n):
        i, j = rng.integers(0, n, 2)
        pairs |= {(i, j), (j, i)}
    rc = np.array(sorted(pairs))
    return rc[:, 0], rc[:, 1]


@pytest.mark.parametrize("transpose", [False, True])
def test_flags_unstable_static_pivot_and_refinement(transpose):
    """Item 0: diagonally dominant (stable in any order); item 1: tiny diagonal entries make the
    static diagonal pivots grow by ~1e12.  The device's backward errors must match the host's
    for the returned solutions, flag item 1 only, and a refinement step must reduce its error."""
    from plate_inverse_problem_amd import _native
    from oracle.plate_oracle import backward_error
    import scipy.sparse as sp
    rng = np.random.default_rng(7)
    n = 96
    rows, cols = _pattern(n, rng)
    solver, r, c = _general_solver(n, rows, cols)
    vals = rng.standard_normal((2, r.size)) + 1j * rng.standard_normal((2, r.size))
    diag = r == c
    vals[0, diag] += 40.0
    vals[1, diag] = 1e-12 * (1 + 1j)                     # every static pivot tiny: large growth
    vals[1, diag & (r % 4 == 0)] = 30.0
    b = rng.standard_normal((2, n)) + 1j * rng.standard_normal((2, n))
    dev = torch.device("cuda", 0)
    data = torch.as_tensor(vals, device=dev)
    bt = torch.as_tensor(b, device=dev)
    out = {}
    for mode in (_native.PFR_CHECK_FORWARD | _native.PFR_CHECK_ADJOINT,
                 _native.PFR_CHECK_FORWARD | _native.PFR_CHECK_ADJOINT | _native.PFR_CHECK_REFINE):
        berr = torch.full((2, 2), float("nan"), dtype=torch.float64, device=dev)
        solver.set_check(mode, 1e-10, berr)
        x = torch.empty_like(bt)
        flags = torch.zeros(2, dtype=torch.int32, device=dev)
        solver.solve(torch.view_as_real(data), r.size, torch.view_as_real(bt), n, torch.view_as_real(x), transpose, 2,
                     flags)
        out[mode] = (x.cpu().numpy(), berr.cpu().numpy()[:, int(transpose)], flags.cpu().numpy())
    bit = _native.PFR_FLAG_BACKWARD_ERROR_ADJ if transpose else _native.PFR_FLAG_BACKWARD_ERROR
    (x0, be0, f0), (x1, be1, f1) = out.values()
    for q in range(2):
        A = sp.csc_matrix((vals[q], (r, c)), shape=(n, n))
        host = backward_error(A, x0[q], b[q], trans=transpose)
        assert be0[q] == pytest.approx(host, rel=0.5, abs=1e-15), (q, be0[q], host)
        assert backward_error(A, x1[q], b[q], trans=transpose) <= max(be1[q] * 2, 1e-15)
    assert be0[0] < 1e-13 and not (f0[0] & bit)
    assert be0[1] > 1e-10 and (f0[1] & bit)
    assert be1[1] < be0[1] * 1e-2                        # one refinement step on the same factors


def test_plate_checks_are_clean_and_match_host():
    """Plate sweeps: forward and adjoint backward errors at machine-precision level, no flags, and
    the device's forward value equals the host's for the oracle's matrices."""
    p = make_problem("orthotropic", ny=5, device="cuda:0")
    freqs = np.linspace(40.0, 600.0, 77)
    fr, berr, flags = p.solveForwardChecked(freqs)
    assert np.all(flags == 0) and berr.max() < 1e-13
    ref = fr * np.exp(0.2j)
    loss = p.getLossFunction(freqs, ref, "MSE_AFC")
    x = torch.tensor(p.parameters * 1.02, requires_grad=True)
    loss(x).backward()
    be = p.engine().last_berr.cpu().numpy()
    assert np.all(np.isfinite(be)) and be.max() < 1e-13 and not p.engine().last_flags.any()


def test_lightly_damped_resonance():
    """beta = 1e-6 (nearly singular at the resonance, condition ~1/beta times the undamped one):
    through the first resonance peak the static-pivot solves stay componentwise backward stable
    (berr at machine precision, nothing flagged), so they agree with the oracle to the conditioning
    (measured 1.4e-6 at the peak, against 1e-9 at beta = 3e-3)."""
    from helpers import make_geometry
    from plate_inverse_problem_amd.Material import get_material
    from plate_inverse_problem_amd.Problem import Problem
    geom, acc = make_geometry(ny=4)
    mat = get_material(7920.0, "isotropic", E=200e9, G=75e9, beta=1e-6)
    p = Problem(geom, mat, acc, device="cuda:0")
    coarse = np.linspace(40.0, 600.0, 2048)
    fc = p.solveForward(coarse)
    k = int(np.argmax(fc))
    fine = np.linspace(coarse[k - 1], coarse[k + 1], 257)
    ff = p.solveForward(fine)
    j = int(np.argmax(ff))
    sel = fine[max(0, j - 2):j + 3]
    fr, berr, flags = p.solveForwardChecked(sel)
    ref = oracle_for(p).fr(sel, p.parameters)
    assert np.all(flags == 0) and berr.max() < 1e-14, (berr, flags)
    assert np.abs(fr / ref - 1).max() < 2e-5, fr / ref - 1
    assert fr.max() > 50 * np.median(fc)                 # the peak is resolved
