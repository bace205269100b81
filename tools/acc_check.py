"""GPU fr against the extended-precision solution of the oracle's fp64 systems, for several
launch-knob settings (read when a solver is created).

    python tools/acc_check.py [ny] [material] [n_freqs] KNOB=V[,KNOB=V] ...
"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")]


def main():
    ny = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    material = sys.argv[2] if len(sys.argv) > 2 else "orthotropic"
    nf = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    cfgs = sys.argv[4:] or [""]
    from make_c3_truth import extended_solve
    from helpers import make_problem, oracle_for
    from oracle.plate_oracle import refined_solve, sparse_lu
    p = make_problem(material, ny=ny)
    orc = oracle_for(p)
    freqs = np.linspace(40.0, 600.0, nf)
    c = orc.coefficients(p.parameters)
    truth, orcl = [], []
    for f in freqs:
        A = orc.matrix(f, c).tocsc()
        A.eliminate_zeros()
        b = (orc.rhs_vec * orc.rhs_scale(f, c)).astype(complex)
        lu = sparse_lu(A)
        truth.append(orc.fr_from_sol(extended_solve(lu, A, b)))
        orcl.append(orc.fr_from_sol(refined_solve(lu, A, b)))
    truth, orcl = np.array(truth), np.array(orcl)
    print("oracle vs truth: max %.2e median %.2e" % (np.max(np.abs(orcl / truth - 1)), np.median(np.abs(orcl / truth - 1))))
    for cfg in cfgs:
        env = dict(kv.split("=") for kv in cfg.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        g = make_problem(material, ny=ny, device="cuda:0")
        fr, berr, flags = g.solveForwardChecked(freqs)
        e = np.abs(fr / truth - 1)
        print("%-30s gpu vs truth: max %.2e median %.2e (at %.1f Hz); max berr %.1e flags %d"
              % (cfg or "default", e.max(), np.median(e), freqs[e.argmax()], berr.max(), int(np.count_nonzero(flags))))
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
