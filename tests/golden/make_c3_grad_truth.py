"""Extended-precision loss + gradient truth over the whole C3 sweep -> ``c3_grad_truth.npz``.

Test data only (run here, committed; ``tests/test_gpu_grad_truth.py`` reads the ``.npz``)::

    python tests/golden/make_c3_grad_truth.py [--workers 8]

The bench's C3 workload (``bench.py``): orthotropic plate, ny = 25 (19,353 DOF), 4,096 frequencies in
40-600 Hz, loss ``MSE_LOG_AFC`` at theta = theta_true (1 + [0.1, 0.1, 0.2, 0.1, 0.1]) against a
synthetic measurement.  For every one of the 4,096 frequencies f the fixture holds

* ``ref``: the measurement, fr at theta_true (phase 0) of the extended-precision solution;
* ``fr_true``: fr at theta of the extended-precision forward solution x;
* ``w_true`` (4096, 18) complex: the frequency's unscaled gradient partials
  ``w_f,k = -lam^T S_k x + e_k lam^T b0`` with ``A^T lam = l'(fr) d fr / d x`` (NON-conjugate
  transpose, ``Sparse.py:211-219`` / ``UMFPACK_Aat`` at ``InnerState.h:183-185``; the adjoint the
  reference's JAX transpose rule solves), contracted in extended precision.  A subset S of the
  frequencies has loss ``sum_S term / |S|`` and partials ``sum_S w_f / |S|``;
* ``fr_oracle``, ``w_oracle``, ``term_oracle``: the same quantities from the fp64 oracle (SuperLU +
  UMFPACK's default refinement, ``oracle.plate_oracle.frequency_partials``) -- the accuracy the
  reference's own refined UMFPACK solves reach, against which the GPU's accuracy is judged.

Extended precision: residuals b - A x and g - A^T lam in numpy ``longdouble`` (64-bit mantissa), the
iterate carried in ``longdouble``, corrections from the fp64 SuperLU factors, until the correction is
below 1e-17 of the iterate or stops shrinking (3-4 steps at C3): the solution of the fp64 matrix to
~cond * 1e-19, orders of magnitude below the fp64 solvers' errors measured against it.
Matrices, right-hand sides and the functional are the oracle's (``oracle/plate_oracle.py``, restating
``Problem.py:437-477``); mesh and material are the bench's (``bench.build_problem``).
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

LD = np.longdouble
_S = {}


def _ld(M):
    r = M.real.astype(LD).tocsr()
    i = M.imag.astype(LD).tocsr()
    return r, i


def ext_solve(lu, A, b, trans=False, max_iter=12):
    """Solution of A x = b (A^T x = b) with residuals in longdouble; returns (xr, xi) longdouble."""
    Ao = A.T.tocsc() if trans else A
    Ar, Ai = _ld(Ao)
    tr = "T" if trans else "N"
    br = np.real(b).astype(LD)
    bi = np.imag(b).astype(LD)
    x0 = lu.solve(np.asarray(b, dtype=complex), trans=tr)
    xr, xi = x0.real.astype(LD), x0.imag.astype(LD)
    return _refine(lu, Ar, Ai, br, bi, xr, xi, tr, max_iter)


def _refine(lu, Ar, Ai, br, bi, xr, xi, tr, max_iter):
    """x += A^{-1} (b - A x) with the residual in longdouble, until the correction is below 1e-17 of x
    or stops shrinking (the longdouble residual's rounding floor)."""
    prev = np.inf
    for it in range(max_iter):
        rr = br - (Ar @ xr - Ai @ xi)
        ri = bi - (Ar @ xi + Ai @ xr)
        d = lu.solve(rr.astype(np.float64) + 1j * ri.astype(np.float64), trans=tr)
        xr += d.real.astype(LD)
        xi += d.imag.astype(LD)
        dn = float(np.max(np.abs(d)))
        xn = float(max(np.max(np.abs(xr)), np.max(np.abs(xi))))
        if dn <= 1e-17 * xn or dn > 0.25 * prev:
            break
        prev = dn
    return xr, xi, it + 1


def _uvw_ld(orc, aU, aV, aW, xr, xi):
    return [(a @ xr, a @ xi) for a in (aU, aV, aW)]


def _worker(idx):
    from oracle.plate_oracle import loss_term_derivative, loss_terms, refined_solve, sparse_lu
    from threadpoolctl import threadpool_limits
    orc, freqs, theta_true, theta, m18, rows, cols, e, rhs = (_S[k] for k in (
        "orc", "freqs", "theta_true", "theta", "m18", "rows", "cols", "e", "rhs"))
    aU, aV, aW = (a.astype(LD) for a in orc.averaging_vectors())
    ts2 = LD(orc.acc_ts) ** 2
    c_true = orc.coefficients(theta_true)
    c = orc.coefficients(theta)
    out = []
    with threadpool_limits(1):
        for i in idx:
            f = freqs[i]
            t0 = time.perf_counter()
            # the measurement: fr at theta_true
            A0 = orc.matrix(f, c_true)
            lu0 = sparse_lu(A0)
            b0 = orc.rhs_vec * orc.rhs_scale(f, c_true)
            xr, xi, _ = ext_solve(lu0, A0, b0)
            (Ur, Ui), (Vr, Vi), (Wr, Wi) = _uvw_ld(orc, aU, aV, aW, xr, xi)
            ref = float(np.sqrt(ts2 * (Ur * Ur + Ui * Ui) + ts2 * (Vr * Vr + Vi * Vi) + Wr * Wr + Wi * Wi))
            # the loss point: forward, fr, cotangent, adjoint, partials -- all extended
            A = orc.matrix(f, c)
            lu = sparse_lu(A)
            b = orc.rhs_vec * orc.rhs_scale(f, c)
            xr, xi, itx = ext_solve(lu, A, b)
            (Ur, Ui), (Vr, Vi), (Wr, Wi) = _uvw_ld(orc, aU, aV, aW, xr, xi)
            fr_ld = np.sqrt(ts2 * (Ur * Ur + Ui * Ui) + ts2 * (Vr * Vr + Vi * Vi) + Wr * Wr + Wi * Wi)
            fr = float(fr_ld)
            # d term / d fr: 2 (log fr - log ref) / fr  (Problem.py:967-975, MSE_LOG_AFC)
            dl = LD(2) * (np.log(fr_ld) - np.log(LD(ref))) / fr_ld
            # g = dl / fr (ts^2 conj(U) aU + ts^2 conj(V) aV + conj(W) aW)
            s = dl / fr_ld
            gr = s * (ts2 * Ur * aU + ts2 * Vr * aV + Wr * aW)
            gi = -s * (ts2 * Ui * aU + ts2 * Vi * aV + Wi * aW)
            # A^T lam = g: first solve on g rounded to fp64, residuals against the longdouble g
            l0 = lu.solve(gr.astype(np.float64) + 1j * gi.astype(np.float64), trans="T")
            Atr, Ati = _ld(A.T.tocsc())
            lr, li, itl = _refine(lu, Atr, Ati, gr, gi, l0.real.astype(LD), l0.imag.astype(LD), "T", 12)
            pr = lr[rows] * xr[cols] - li[rows] * xi[cols]
            pi = lr[rows] * xi[cols] + li[rows] * xr[cols]
            tr_ = lr @ rhs
            ti_ = li @ rhs
            wr = -(m18 @ pr) + e * tr_
            wi = -(m18 @ pi) + e * ti_
            w = wr.astype(np.float64) + 1j * wi.astype(np.float64)
            term = float((np.log(fr_ld) - np.log(LD(ref))) ** 2)
            # the fp64 oracle at the same frequency (refined SuperLU, its own contraction)
            xo = refined_solve(lu, A, b)
            Uo, Vo, Wo = (a.astype(np.float64) @ xo for a in (aU, aV, aW))
            t2 = float(orc.acc_ts) ** 2
            fro = float(np.sqrt(t2 * abs(Uo) ** 2 + t2 * abs(Vo) ** 2 + abs(Wo) ** 2))
            dlo = float(loss_term_derivative(fro, ref, "MSE_LOG_AFC"))
            go = (dlo / fro) * (t2 * np.conj(Uo) * aU.astype(np.float64) + t2 * np.conj(Vo) * aV.astype(np.float64)
                                + np.conj(Wo) * aW.astype(np.float64))
            lo = refined_solve(lu, A, go, trans=True)
            po = lo[rows] * xo[cols]
            m64 = _S["m18_64"]
            wo = -(m64 @ po.real + 1j * (m64 @ po.imag)) + _S["e64"] * (lo @ orc.rhs_vec)
            termo = float(loss_terms(fro, ref, "MSE_LOG_AFC"))
            out.append((i, ref, fr, term, w, fro, termo, wo, itx, itl))
            print(f"{i:5d} {f:8.3f} Hz fr {fr:.6e} oracle fr {abs(fro / fr - 1):.1e} w {np.max(np.abs(wo - w)) / np.max(np.abs(w)):.1e}"
                  f" iters {itx}/{itl} {time.perf_counter() - t0:.1f} s", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--n", type=int, default=4096, help="sweep size (the fixture: 4096)")
    ap.add_argument("--only", type=int, default=0, help="debug: only this many frequencies")
    args = ap.parse_args()
    import multiprocessing as mp
    from helpers import make_problem, oracle_for
    from oracle.plate_oracle import RHS_WEIGHTS_D
    p = make_problem("orthotropic", ny=25)
    orc = oracle_for(p)
    theta_true = np.asarray(p.parameters, dtype=np.float64)
    theta = theta_true * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1]))
    freqs = np.linspace(40.0, 600.0, args.n)
    e = np.concatenate([np.zeros(12), RHS_WEIGHTS_D])
    _S.update(orc=orc, freqs=freqs, theta_true=theta_true, theta=theta, m18=orc.mats[:18].astype(LD),
              m18_64=orc.mats[:18], rows=orc.rows.astype(np.int64), cols=orc.cols.astype(np.int64),
              e=e.astype(LD), e64=e, rhs=orc.rhs_vec.astype(LD))
    todo = np.arange(args.n) if not args.only else np.linspace(0, args.n - 1, args.only).round().astype(int)
    chunks = [c for c in np.array_split(todo, args.workers * 8) if c.size]
    t0 = time.perf_counter()
    with mp.get_context("fork").Pool(args.workers) as pool:
        res = [r for part in pool.imap_unordered(_worker, chunks) for r in part]
    res.sort(key=lambda r: r[0])
    idx = np.array([r[0] for r in res])
    print(f"{len(res)} frequencies in {time.perf_counter() - t0:.0f} s", flush=True)
    name = "c3_grad_truth.npz" if not args.only else "c3_grad_truth_debug.npz"
    np.savez_compressed(
        os.path.join(HERE, name), material="orthotropic", ny=25, n_sweep=args.n, index=idx, freqs=freqs[idx],
        theta_true=theta_true, theta=theta, loss="MSE_LOG_AFC",
        ref=np.array([r[1] for r in res]), fr_true=np.array([r[2] for r in res]),
        term_true=np.array([r[3] for r in res]), w_true=np.array([r[4] for r in res]),
        fr_oracle=np.array([r[5] for r in res]), term_oracle=np.array([r[6] for r in res]),
        w_oracle=np.array([r[7] for r in res]), iters=np.array([(r[8], r[9]) for r in res]))


if __name__ == "__main__":
    main()
