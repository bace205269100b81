"""CPU ORACLE for the plate frequency-response hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``plate_inverse_problem_amd``) never imports it; it fails
loudly when its HIP library is missing.

A numpy/scipy restatement of the reference's per-frequency computation:

* ``abd_transform``  -- ``source/jax_plate/Material.py:372-391`` (isotropic),
  ``:455-482`` (orthotropic), ``:571-602`` (orthotropic_d4), ``:743-764`` (sol),
  ``:812-833`` (symm_sol);
* ``inertia``        -- ``Problem.py:356-374``;
* ``assemble``       -- ``Problem.py:437-445``;
* ``rhs``            -- ``Problem.py:447-449``;
* solve              -- ``Problem.py:452`` -> ``Sparse.py:231`` ->
  ``InnerState.h:276-288`` (UMFPACK numeric+solve per frequency).  UMFPACK is
  not available; this oracle uses scipy SuperLU (complex128, threshold partial
  pivoting) followed by UMFPACK's default iterative refinement (the reference
  passes a NULL Control, so ``umfpack_zi_solve`` refines up to UMFPACK_IRSTEP = 2
  steps, ``refined_solve``).  UMFPACK itself cannot be built here and no reference
  test pins solver outputs; the restatement is pinned against the
  reference's own Problem / Optimizers code run with this solve in UMFPACK's place
  (``reference_run.npz``, below) and by a dense ``numpy.linalg.solve`` cross-check;
* ``functional``     -- ``Problem.py:454-477`` (dense interpolation, means,
  ``fr = sqrt((ts|U|)^2 + (ts|V|)^2 + |W|^2)``);
* ``loss``           -- ``Problem.py:948-975`` (MSE, RMSE, MSE_AFC, MSE_LOG_AFC);
* ``loss_and_grad``  -- reverse mode through the solve as JAX does it with the
  reference primitives: transpose of ``spsolve`` is a solve with the
  NON-conjugate transpose (``Sparse.py:211-219``, ``UMFPACK_Aat`` at
  ``InnerState.h:183-185``); the matrix cotangent is ``ct[row] * x[col]``
  (``Sparse.py:173-176``).

Pins of the restatement itself: ``tests/golden/reference_run.npz`` -- outputs of
the reference's own ``Problem.solveForward`` / ``getLossFunction`` (4 losses) /
``Optimizers.optimize_gd`` / ``optimize_cd`` run here on CPU under numpy stand-ins
for JAX (``tests/golden/make_reference_run.py``; the only non-reference arithmetic
in that chain is this module's ``refined_solve`` standing in for UMFPACK),
``tests/golden/material_abd.json`` (reference ``Material.py`` outputs),
``tests/golden/layout_*.npz`` / ``freefem_stream.npz`` (reference block layout and
FreeFEM stream parsers), extended-precision truth fixtures at C2 / C3 size
(``tests/golden/make_c3_truth.py``), finite differences and a dense-solve
cross-check (tests/).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

LOSS_TYPES = ("MSE", "RMSE", "MSE_AFC", "MSE_LOG_AFC")
RHS_WEIGHTS_D = np.array([1.0, 2.0, 4.0, 1.0, 4.0, 4.0])   # Problem.py:447-448: D0+2D1+4D2+D3+4D4+4D5


# ----------------------------------------------------------------------------- transforms
def _laminate_maps(angles, h):
    """Numeric Q->ABD maps of ``Material.py:660-741`` (independent restatement)."""
    ang = np.deg2rad(np.asarray(angles, dtype=np.float64))
    n = ang.size
    z = np.linspace(-h / 2, h / 2, n + 1)
    comps = [(0, 0), (0, 1), (0, 2), (1, 1), (1, 2), (2, 2)]
    out = np.zeros((3, 6, 6))
    for k in range(n):
        c, s = np.cos(ang[k]), -np.sin(ang[k])
        T = np.array([[c * c, s * s, -2 * c * s], [s * s, c * c, 2 * c * s], [c * s, -c * s, c * c - s * s]])
        dz = [z[k + 1] - z[k], (z[k + 1] ** 2 - z[k] ** 2) / 2, (z[k + 1] ** 3 - z[k] ** 3) / 3]
        for j, (a, b) in enumerate(comps):
            if j in (2, 4):
                continue
            Q = np.zeros((3, 3))
            Q[a, b] = Q[b, a] = 1.0
            QT = T @ Q @ T.T
            for i, (p, q) in enumerate(comps):
                for m in range(3):
                    out[m, i, j] += QT[p, q] * dz[m]
    return out


def abd_transform(atype: str, h: float, theta, angles=None):
    """theta -> (A, B, D), complex (6,) each, order 11, 12, 16, 22, 26, 66."""
    t = np.asarray(theta, dtype=np.float64)
    if atype == "isotropic":
        E, G, beta = t
        nu = E / (2 * G) - 1
        A = E * h / (1 - nu ** 2)
        D = A * h ** 2 / 12
        arr = np.array([1.0, nu, 0.0, 1.0, 0.0, (1 - nu) / 2]) * (1 + 1j * beta)
        return A * arr, np.zeros(6, complex), D * arr
    if atype in ("orthotropic", "orthotropic_d4"):
        if atype == "orthotropic":
            E1, E2, G12, nu12 = t[:4]
            lf = 1 + 1j * t[4]
        else:
            E1, E2, G12, nu12 = (t[i] * (1 + 1j * t[4 + i]) for i in range(4))
            lf = 1.0
        r = E2 / E1
        nu21 = r * nu12
        A11 = E1 * h / (1 - nu12 * nu21)
        D11 = E1 * h ** 3 / (12 * (1 - nu12 * nu21))
        As = np.array([A11, nu21 * A11, 0, r * A11, 0, G12 * h], dtype=complex) * lf
        Ds = np.array([D11, nu21 * D11, 0, D11 / r, 0, G12 * h ** 3 / 12], dtype=complex) * lf
        return As, np.zeros(6, complex), Ds
    if atype in ("sol", "symm_sol"):
        if atype == "symm_sol":
            E1, G12, nu12, beta = t
            E2 = E1
        else:
            E1, E2, G12, nu12, beta = t
        den = 1 - E2 / E1 * nu12 ** 2
        Q = np.array([E1 / den, nu12 * E2 / den, 0, E2 / den, 0, G12])
        M = _laminate_maps(angles, h)
        A, B, D = ((M[k] @ Q) * (1 + 1j * beta) for k in range(3))
        a = np.asarray(angles, dtype=np.float64)
        if np.sum(np.abs(a - a[::-1])) <= 1e-6:
            B = np.zeros(6, complex)      # exact zero of the reference's sympy integration
        return A, B, D
    raise ValueError(atype)


def _mr(M, z):
    """real matrix @ complex vector via two real BLAS calls (numpy's mixed-dtype
    matmul takes a slow non-BLAS loop)."""
    return M @ z.real + 1j * (M @ z.imag)


def _rc(c, M):
    """complex vector @ real matrix."""
    return c.real @ M + 1j * (c.imag @ M)


def sparse_lu(A):
    """SuperLU with a diagonal-preferring threshold (0.001), like UMFPACK's
    symmetric strategy; partial pivoting (threshold 1.0) on these FE matrices
    picks off-diagonal pivots and fills in 10x more (measured)."""
    A = A.tocsc(copy=True)             # eliminate_zeros works in place: never on the caller's arrays
    A.eliminate_zeros()
    return spla.splu(A, permc_spec="COLAMD", diag_pivot_thresh=0.001, options=dict(SymmetricMode=True))


IR_STEPS = 2                       # UMFPACK default Control[UMFPACK_IRSTEP]
EPS = np.finfo(np.float64).eps


def backward_error(A, x, b, trans=False):
    """Componentwise (Oettli-Prager) backward error max_i |b - A x|_i / (|A| |x| + |b|)_i, the
    sparse backward error UMFPACK's refinement monitors (its omega1; rows with a zero
    denominator count as exact when their residual is zero, infinite otherwise)."""
    Ao = A.T if trans else A
    r = np.abs(b - Ao @ x)
    den = abs(Ao) @ np.abs(x) + np.abs(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        w = np.where(den > 0, r / np.where(den > 0, den, 1.0), np.where(r > 0, np.inf, 0.0))
    return float(w.max()) if w.size else 0.0


def refined_solve(lu, A, b, trans=False, steps=IR_STEPS):
    """``umfpack_zi_solve`` with the default Control (InnerState.h:246-247 passes NULL):
    the solve followed by up to UMFPACK_IRSTEP = 2 steps of iterative refinement on the
    same factors, x += A^{-1}(b - A x) (A^T for the non-conjugate transpose, UMFPACK_Aat),
    stopped once the sparse backward error reaches machine precision or stops halving
    (the better iterate is kept).  Without it an fp64 LU of these badly scaled systems
    (membrane, bending and unit Dirichlet rows) is off by up to ~4e-5 in fr at the C3
    size."""
    tr = "T" if trans else "N"
    b = np.asarray(b, dtype=complex)
    x = lu.solve(b, trans=tr)
    om = backward_error(A, x, b, trans)
    for _ in range(steps):
        if om <= EPS:
            break
        r = b - (A.T @ x if trans else A @ x)
        xn = x + lu.solve(r, trans=tr)
        omn = backward_error(A, xn, b, trans)
        if omn > om / 2:
            if omn < om:
                x, om = xn, omn
            break
        x, om = xn, omn
    return x


def coeffs18(atype, h, theta, angles=None):
    A, B, D = abd_transform(atype, h, theta, angles)
    return np.concatenate([A, B, D])


def coeffs18_jacobian(atype, h, theta, angles=None):
    """d c_k / d theta_p by 4th-order central differences, (18, n_theta) complex."""
    t = np.asarray(theta, dtype=np.float64)
    J = np.zeros((18, t.size), dtype=complex)
    for p in range(t.size):
        step = 1e-4 * max(abs(t[p]), 1e-12)
        vals = []
        for m in (-2, -1, 1, 2):
            tt = t.copy()
            tt[p] += m * step
            vals.append(coeffs18(atype, h, tt, angles))
        J[:, p] = (vals[0] - 8 * vals[1] + 8 * vals[2] - vals[3]) / (12 * step)
    return J


def inertia(h, rho, acc_mass, acc_radius, acc_height):
    """(I0, I0Corr, I2, I2Corr), Problem.py:356-374."""
    rho_c = acc_mass / (np.pi * acc_radius ** 2) / acc_height
    return (h * rho, acc_height * rho_c, rho * h ** 3 / 12,
            rho_c / 3 * ((h / 2 + acc_height) ** 3 - h ** 3 / 8))


# ----------------------------------------------------------------------------- problem data
@dataclass
class OracleProblem:
    n: int
    rows: np.ndarray            # (nnz,) CSC-ordered coordinates of the union pattern
    cols: np.ndarray
    mats: np.ndarray            # (26, nnz) float64
    rhs_vec: np.ndarray         # (n,)
    IL: np.ndarray              # (P, Lh) dense
    IM: np.ndarray              # (P, Mh)
    IWx: np.ndarray
    IWy: np.ndarray
    Lh: int
    I: tuple                    # (I0, I0Corr, I2, I2Corr)
    acc_h: float
    acc_h_eff: float
    acc_ts: float
    atype: str
    h: float
    angles: object = None

    # -- assembly (Problem.py:437-449) --
    def coefficients(self, theta):
        return coeffs18(self.atype, self.h, theta, self.angles)

    def mass_values(self):
        m = self.mats
        I0, I0c, I2, I2c = self.I
        return I0 * (m[18] + m[20] + m[22]) + I0c * (m[19] + m[21] + m[23]) + I2 * m[24] + I2c * m[25]

    def matrix(self, f, c):
        """A(omega) on the CSC union pattern (rows/cols are already in CSC order)."""
        if not hasattr(self, "_csc"):
            colptr = np.zeros(self.n + 1, dtype=np.int64)
            np.add.at(colptr, self.cols.astype(np.int64) + 1, 1)
            self._csc = (self.rows.astype(np.int32), np.cumsum(colptr).astype(np.int32), self.mass_values())
        rowind, colptr, mass = self._csc
        omega = 2 * np.pi * f
        data = -omega ** 2 * mass + _rc(c, self.mats[:18])
        return sp.csc_matrix((data, rowind.copy(), colptr.copy()), shape=(self.n, self.n))

    def rhs_scale(self, f, c):
        omega = 2 * np.pi * f
        return RHS_WEIGHTS_D @ c[12:18] - omega ** 2 * sum(self.I)

    # -- functional (Problem.py:454-477) --
    def uvw(self, sol):
        L = self.Lh
        u_sol = _mr(self.IL, sol[:L])
        v_sol = _mr(self.IL, sol[L:2 * L])
        w_sol = _mr(self.IM, sol[2 * L:])
        wx_sol = _mr(self.IWx, sol[2 * L:])
        wy_sol = _mr(self.IWy, sol[2 * L:])
        k = self.acc_h_eff * self.acc_h
        return np.mean(u_sol - k * wx_sol), np.mean(v_sol - k * wy_sol), np.mean(w_sol)

    def fr_from_sol(self, sol):
        U, V, W = self.uvw(sol)
        ts = self.acc_ts
        return np.sqrt((np.abs(U) * ts) ** 2 + (np.abs(V) * ts) ** 2 + np.abs(W) ** 2)

    def averaging_vectors(self):
        """(aU, aV, aW) with U = aU . x etc. -- used for the adjoint seed."""
        L, n = self.Lh, self.n
        k = self.acc_h_eff * self.acc_h
        P = self.IL.shape[0]
        aU = np.zeros(n)
        aV = np.zeros(n)
        aW = np.zeros(n)
        aU[:L] = self.IL.sum(0) / P
        aU[2 * L:] = -k * self.IWx.sum(0) / P
        aV[L:2 * L] = self.IL.sum(0) / P
        aV[2 * L:] = -k * self.IWy.sum(0) / P
        aW[2 * L:] = self.IM.sum(0) / P
        return aU, aV, aW

    # -- per-frequency solves --
    def solve(self, f, theta):
        c = self.coefficients(theta)
        A = self.matrix(f, c)
        b = self.rhs_vec * self.rhs_scale(f, c)
        lu = sparse_lu(A)
        return refined_solve(lu, A, b), lu, A

    def fr(self, freqs, theta):
        return np.array([self.fr_from_sol(self.solve(f, theta)[0]) for f in np.asarray(freqs)])

    def solutions(self, freqs, theta):
        return np.stack([self.solve(f, theta)[0] for f in np.asarray(freqs)])


def loss_terms(fr, ref, loss_type):
    """Per-frequency terms whose mean is the loss (Problem.py:948-975)."""
    fr = np.asarray(fr, dtype=np.float64)
    ref = np.asarray(ref)
    if loss_type == "MSE":
        return np.abs(fr - ref) ** 2
    if loss_type == "RMSE":
        return np.abs((fr - ref) / ref) ** 2
    if loss_type == "MSE_AFC":
        return (np.abs(fr) - np.abs(ref)) ** 2
    if loss_type == "MSE_LOG_AFC":
        return (np.log(np.abs(fr)) - np.log(np.abs(ref))) ** 2
    raise ValueError(loss_type)


def loss_term_derivative(fr, ref, loss_type):
    """d(term)/d(fr) for real fr > 0."""
    fr = np.asarray(fr, dtype=np.float64)
    ref = np.asarray(ref)
    if loss_type == "MSE":
        return 2 * (fr - ref.real)
    if loss_type == "RMSE":
        return 2 * (fr - ref.real) / np.abs(ref) ** 2
    if loss_type == "MSE_AFC":
        return 2 * (fr - np.abs(ref))
    if loss_type == "MSE_LOG_AFC":
        return 2 * (np.log(fr) - np.log(np.abs(ref))) / fr
    raise ValueError(loss_type)


def loss(prob: OracleProblem, freqs, ref, loss_type, theta):
    return float(np.mean(loss_terms(prob.fr(freqs, theta), ref, loss_type)))


def frequency_partials(prob: OracleProblem, freqs, ref, loss_type, theta, n_total=None,
                       refactor_adjoint=False, factorisations=None):
    """Per-chunk partial sums (loss_sum, w (18,) complex) -- the quantity the
    GPU sweep reduces and ranks all-reduce.  ``w_k = sum_f (-lam^T m_k x + e_k lam^T b0)``.
    ``refactor_adjoint=True`` refactorises for the adjoint solve like the
    reference's transpose bind (InnerState.h:276-288); ``factorisations=n`` (n >= 2)
    runs the reference's full count per frequency: the primal factorisation, then
    n - 1 transposed binds, each with a fresh factorisation (Sparse.py:211-222 binds
    ``spsolve(..., transpose=True)`` once per cotangent branch, and every bind
    factorises, InnerState.h:276-288) -- the repeated
    adjoints are identical, only the count of work differs."""
    freqs = np.asarray(freqs, dtype=np.float64)
    ref = np.asarray(ref)
    n_total = freqs.size if n_total is None else n_total
    c = prob.coefficients(theta)
    aU, aV, aW = prob.averaging_vectors()
    ts2 = prob.acc_ts ** 2
    e = np.concatenate([np.zeros(12), RHS_WEIGHTS_D])
    w = np.zeros(18, dtype=complex)
    loss_sum = 0.0
    rows, cols, m18 = prob.rows, prob.cols, prob.mats[:18]
    n_fact = factorisations or (2 if refactor_adjoint else 1)
    for i, f in enumerate(freqs):
        A = prob.matrix(f, c)
        lu = sparse_lu(A)
        x = refined_solve(lu, A, prob.rhs_vec * prob.rhs_scale(f, c))
        U, V, W = aU @ x, aV @ x, aW @ x
        fr = np.sqrt(ts2 * abs(U) ** 2 + ts2 * abs(V) ** 2 + abs(W) ** 2)
        loss_sum += float(loss_terms(fr, ref[i], loss_type))
        dl = float(loss_term_derivative(fr, ref[i], loss_type)) / n_total
        g = (dl / fr) * (ts2 * np.conj(U) * aU + ts2 * np.conj(V) * aV + np.conj(W) * aW)
        if n_fact == 1:
            lam = refined_solve(lu, A, g, trans=True)
        for _ in range(n_fact - 1):
            lam = refined_solve(sparse_lu(A), A, g, trans=True)
        p = lam[rows] * x[cols]
        w += -_mr(m18, p) + e * (lam @ prob.rhs_vec)
    return loss_sum, w


def loss_and_grad(prob: OracleProblem, freqs, ref, loss_type, theta, scaling=None):
    """(loss, dloss/dtheta) by the adjoint method; theta may be scaled as in
    ``getLossFunction(..., scaling_params)`` (Problem.py:943-950)."""
    theta = np.asarray(theta, dtype=np.float64)
    s = np.ones_like(theta) if scaling is None else np.asarray(scaling, dtype=np.float64)
    phys = theta * s
    loss_sum, w = frequency_partials(prob, freqs, ref, loss_type, phys)
    J = coeffs18_jacobian(prob.atype, prob.h, phys, prob.angles)
    grad = np.real(w @ J) * s
    return loss_sum / np.asarray(freqs).size, grad


def fd_grad(prob: OracleProblem, freqs, ref, loss_type, theta, rel=2e-4):
    """4th-order central differences (truncation O(h^4): the loss is sharply
    peaked in the loss factor near resonances, O(h^2) stencils are not enough)."""
    theta = np.asarray(theta, dtype=np.float64)
    g = np.zeros_like(theta)
    for p in range(theta.size):
        h = rel * abs(theta[p])
        v = []
        for m in (-2, -1, 1, 2):
            t = theta.copy()
            t[p] += m * h
            v.append(loss(prob, freqs, ref, loss_type, t))
        g[p] = (v[0] - 8 * v[1] + 8 * v[2] - v[3]) / (12 * h)
    return g


# ----------------------------------------------------------------------------- CPU baseline
_POOL_PROB = None


def _pool_worker(args):
    # one process per core: keep BLAS single-threaded (oversubscription otherwise
    # multiplies the run time many-fold on a cgroup-limited host)
    from threadpoolctl import threadpool_limits
    freqs, ref, loss_type, theta, n_total, refactor, nfact = args
    with threadpool_limits(1):
        return frequency_partials(_POOL_PROB, freqs, ref, loss_type, theta, n_total, refactor, nfact)


def parallel_partials(prob: OracleProblem, freqs, ref, loss_type, theta, n_workers=None,
                      refactor_adjoint=False, factorisations=None):
    """Process-pool CPU sweep (SuperLU holds the GIL, so processes, not threads).
    Returns (loss_sum, w, n_workers)."""
    import multiprocessing as mp
    global _POOL_PROB
    n_workers = n_workers or os.cpu_count() or 1
    freqs = np.asarray(freqs)
    ref = np.asarray(ref)
    chunks = [c for c in np.array_split(np.arange(freqs.size), n_workers) if c.size]
    _POOL_PROB = prob
    ctx = mp.get_context("fork")
    with ctx.Pool(len(chunks)) as pool:
        parts = pool.map(_pool_worker, [(freqs[c], ref[c], loss_type, theta, freqs.size, refactor_adjoint,
                                         factorisations) for c in chunks])
    _POOL_PROB = None
    return sum(p[0] for p in parts), sum(p[1] for p in parts), len(chunks)
