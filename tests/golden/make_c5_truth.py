"""Extended-precision losses along the C5 L-BFGS trajectory -> ``c5_truth.npz``.

Test data only (run here, committed; ``tests/test_gpu_c5.py`` reads the ``.npz``)::

    python tests/golden/make_c5_truth.py

C5 (BASELINE.json configs[4]): L-BFGS over the 8 parameters of ``orthotropic_d4`` on the C3 mesh (ny = 25,
19,353 DOF), loss MSE_LOG_AFC, scaled parameters x = theta / theta0 from the start of ``tools/c5_lbfgs.py``.
On the 32-frequency subsample the GPU test uses (every 128th of linspace(40, 600, 4096)):
* the reference FR: the extended-precision fr at theta_true (phase 0, as ``Problem.py:207``);
* the trajectory: 3 L-BFGS steps of this build's ``Optimizers.optimize_lbfgs`` driven by the oracle's loss and
  adjoint gradient (SuperLU + UMFPACK-default refinement, ``tests/oracle_loss.py``), so the iterates do not
  depend on the GPU;
* at every iterate: the loss from fr solved with residuals in extended precision (numpy ``longdouble``) on the
  SuperLU factors until converged (``make_c3_truth.extended_solve``), and the fp64 oracle's loss beside it.
The GPU test evaluates its loss at the same iterates and compares it with the extended-precision loss.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), HERE]

from helpers import make_problem, oracle_for  # noqa: E402
from make_c3_truth import extended_solve  # noqa: E402
from oracle.plate_oracle import loss_terms, refined_solve, sparse_lu  # noqa: E402

REL0 = np.array([0.02, -0.02, 0.03, 0.01, 0.05, -0.05, 0.04, 0.03])     # tools/c5_lbfgs.py start
_ORC = None


def _fr_pair(args):
    f, theta = args
    from threadpoolctl import threadpool_limits
    with threadpool_limits(1):
        c = _ORC.coefficients(theta)
        A = _ORC.matrix(f, c).tocsc()
        A.eliminate_zeros()
        b = (_ORC.rhs_vec * _ORC.rhs_scale(f, c)).astype(complex)
        lu = sparse_lu(A)
        return _ORC.fr_from_sol(extended_solve(lu, A, b)), _ORC.fr_from_sol(refined_solve(lu, A, b))


def fr_truth(orc, freqs, theta, workers=8):
    """(extended-precision fr, fp64 oracle fr) at theta, one process per frequency chunk."""
    import multiprocessing as mp
    global _ORC
    _ORC = orc
    with mp.get_context("fork").Pool(workers) as pool:
        out = pool.map(_fr_pair, [(f, np.asarray(theta, dtype=np.float64)) for f in freqs])
    return np.array([o[0] for o in out]), np.array([o[1] for o in out])


def main():
    import torch
    from oracle_loss import oracle_loss_fn
    from plate_inverse_problem_amd import Optimizers
    p = make_problem("orthotropic_d4", ny=25)
    orc = oracle_for(p)
    freqs = np.linspace(40.0, 600.0, 4096)[::128]
    theta_true = np.asarray(p.parameters, dtype=np.float64)
    ref = fr_truth(orc, freqs, theta_true)[0].astype(np.complex128)
    th0 = theta_true * (1 + REL0)
    orc_fn = oracle_loss_fn(orc, freqs, ref, "MSE_LOG_AFC", scaling=th0, n_workers=8)
    res = Optimizers.optimize_lbfgs(orc_fn, np.ones(8), N_steps=3)
    X = np.array([np.asarray(v, dtype=np.float64) for v in res.x_history + [res.x]])
    loss_true, loss_orc, frs = [], [], []
    for x in X:
        ft, fo = fr_truth(orc, freqs, x * th0)
        frs.append(ft)
        loss_true.append(float(np.mean(loss_terms(ft, ref, "MSE_LOG_AFC"))))
        loss_orc.append(float(np.mean(loss_terms(fo, ref, "MSE_LOG_AFC"))))
        print(f"x {np.array2string(x, precision=6)} loss {loss_true[-1]:.15e} oracle rel "
              f"{abs(loss_orc[-1] / loss_true[-1] - 1):.2e}", flush=True)
    np.savez_compressed(os.path.join(HERE, "c5_truth.npz"), material="orthotropic_d4", ny=25, freqs=freqs, ref=ref,
                        theta_true=theta_true, theta0=th0, x=X, loss_true=np.array(loss_true),
                        loss_oracle=np.array(loss_orc), fr_true=np.array(frs))
    del torch


if __name__ == "__main__":
    main()
