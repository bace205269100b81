"""Extended-precision reference solutions at the benchmark sizes -> ``c3_truth.npz``, ``c2_truth.npz``.

Test data only (run here, committed; the GPU tests read the ``.npz``)::

    python tests/golden/make_c3_truth.py

At the C3 size (orthotropic, ny = 25, 19,353 DOF) the plate systems are badly scaled (membrane,
bending and unit Dirichlet rows) and ill-conditioned: an fp64 sparse LU with threshold pivoting
(SuperLU, COLAMD, diagonal threshold 0.001) is off by up to 4e-5 in fr, although its normwise
backward error is 1e-15 (its componentwise backward error is 1e-9).  The fixture holds, per
frequency, fr of the solution refined with residuals in extended precision (numpy ``longdouble``,
64-bit mantissa) on the SuperLU factors until converged -- the exact solution of the oracle's fp64
matrix to ~1e-13 -- next to the fp64 oracle (SuperLU + UMFPACK-style refinement,
``oracle.plate_oracle.refined_solve``).  Matrices, right-hand sides and the FR functional are the
oracle's (``oracle/plate_oracle.py``, restating ``Problem.py:437-477``); mesh and material are the
bench's (``bench.build_problem``) at theta_true.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from helpers import make_problem, oracle_for  # noqa: E402
from oracle.plate_oracle import backward_error, refined_solve, sparse_lu  # noqa: E402


def extended_solve(lu, A, b, iters=8):
    """x with b - A x evaluated in longdouble, corrections from the fp64 factors (converged when
    cond * eps < 1; the iterate is carried in longdouble)."""
    Ar = A.real.astype(np.longdouble).tocsr()
    Ai = A.imag.astype(np.longdouble).tocsr()
    br, bi = b.real.astype(np.longdouble), b.imag.astype(np.longdouble)
    x0 = lu.solve(b)
    xr, xi = x0.real.astype(np.longdouble), x0.imag.astype(np.longdouble)
    for _ in range(iters):
        rr = br - (Ar @ xr - Ai @ xi)
        ri = bi - (Ar @ xi + Ai @ xr)
        d = lu.solve(rr.astype(np.float64) + 1j * ri.astype(np.float64))
        xr += d.real.astype(np.longdouble)
        xi += d.imag.astype(np.longdouble)
    return xr.astype(np.float64) + 1j * xi.astype(np.float64)


def make(name, material, ny, n_sweep, peak_idx):
    p = make_problem(material, ny=ny)
    orc = oracle_for(p)
    sweep = np.linspace(40.0, 600.0, n_sweep)
    idx = np.unique(np.concatenate([np.linspace(0, n_sweep - 1, 29).round().astype(int), np.asarray(peak_idx, dtype=int)]))
    freqs = sweep[idx]
    c = orc.coefficients(p.parameters)
    fr_true, fr_orc, fr_lu, berr_lu = [], [], [], []
    for f in freqs:
        A = orc.matrix(f, c).tocsc()
        A.eliminate_zeros()
        b = (orc.rhs_vec * orc.rhs_scale(f, c)).astype(complex)
        lu = sparse_lu(A)
        x_lu = lu.solve(b)
        fr_true.append(orc.fr_from_sol(extended_solve(lu, A, b)))
        fr_orc.append(orc.fr_from_sol(refined_solve(lu, A, b)))
        fr_lu.append(orc.fr_from_sol(x_lu))
        berr_lu.append(backward_error(A, x_lu, b))
        print(f"{name} {f:8.3f} Hz fr {fr_true[-1]:.15e}  oracle {abs(fr_orc[-1] / fr_true[-1] - 1):.1e}  "
              f"unrefined LU {abs(fr_lu[-1] / fr_true[-1] - 1):.1e} (berr {berr_lu[-1]:.1e})", flush=True)
    np.savez_compressed(os.path.join(HERE, f"{name}_truth.npz"), material=material, ny=ny, n_sweep=n_sweep,
                        index=idx, freqs=freqs, theta=np.asarray(p.parameters), fr_true=np.array(fr_true),
                        fr_oracle=np.array(fr_orc), fr_unrefined=np.array(fr_lu), berr_unrefined=np.array(berr_lu))


if __name__ == "__main__":
    which = sys.argv[1:] or ["c3", "c2"]
    # peak indices: the resonance maxima of the GPU sweeps (C3: sample 1179 of 4096 = 201.23 Hz)
    if "c3" in which:
        make("c3", "orthotropic", 25, 4096, [1178, 1179, 1180])
    if "c2" in which:
        make("c2", "isotropic", 12, 1024, [])
