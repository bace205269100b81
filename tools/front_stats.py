"""Per-level front statistics of the C3 symbolic analysis (CPU only, no GPU needed).

Usage: python tools/front_stats.py [ny]
Prints per level: fronts, pivots, max front, algorithmic Schur bytes (A22 lower stores + L21
read once) and the operand bytes the 4 x 4 Schur tiles load from L2 (9 loads per pivot step),
both per frequency.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import build_problem  # noqa: E402
from plate_inverse_problem_amd import _native  # noqa: E402
from plate_inverse_problem_amd.Problem import KB_SLICE, decoupled_symmetric  # noqa: E402


def symbolic(p):
    mats = p.mats
    active = [k for k in range(26) if not (p.material.is_mps and KB_SLICE.start <= k < KB_SLICE.stop)]
    keep = np.nonzero(p.present[active].any(axis=0) & (mats[active] != 0).any(axis=0))[0]
    rows, cols = p.rows[keep], p.cols[keep]
    n = p.mat_size
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(colptr, cols.astype(np.int64) + 1, 1)
    colptr = np.cumsum(colptr).astype(np.int32)
    sym = decoupled_symmetric(rows, cols, mats[:, keep], n)
    return _native.Symbolic(n, colptr, rows.astype(np.int32), symmetric=sym), sym


def main(ny):
    p = build_problem(ny, "cpu")
    S, sym = symbolic(p)
    fr = S.export("FRONTS").reshape(-1, 8)
    ns, f, lvl = fr[:, 0], fr[:, 1], fr[:, 5]
    r = f - ns
    print("symmetric", sym, S.stats())
    print("%3s %6s %7s %5s %5s %9s %9s %6s" % ("lvl", "fronts", "pivots", "maxf", "maxns", "alg MB", "L2ld MB", "ratio"))
    T = [0, 0]
    for l in range(int(lvl.max()) + 1):
        m = lvl == l
        rr, nn = r[m], ns[m]
        alg = 16 * (rr * (rr + 1) // 2 + rr * nn).sum()
        tiles = sum(sum(1 for i0 in range(0, x, 4) for j0 in range(0, min(x, i0 + 4), 4)) for x in rr)
        ld = 0
        for x, k in zip(rr, nn):
            nt = sum(1 for i0 in range(0, x, 4) for j0 in range(0, min(x, i0 + 4), 4))
            ld += nt * (9 * k + 32) * 16
        T[0] += alg
        T[1] += ld
        print("%3d %6d %7d %5d %5d %9.2f %9.2f %6.1f  tiles %d" % (l, m.sum(), nn.sum(), f[m].max(), nn.max(),
                                                                alg / 1e6, ld / 1e6, ld / max(alg, 1), tiles))
    print("total alg %.2f MB, L2 operand loads %.2f MB per frequency" % (T[0] / 1e6, T[1] / 1e6))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 25)
