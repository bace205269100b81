"""Numpy model of the HIP multifrontal algorithm, driven by the C-ABI's exported
symbolic maps (test infrastructure: validates the host symbolic analysis on
CPU, without a GPU).  Mirrors csrc/kernels.hip phase by phase, for ONE matrix.
"""
from __future__ import annotations

import numpy as np


class MFModel:
    def __init__(self, sym):
        self.fr = sym.export("FRONTS")           # ns, f, row0, col0, parent, level, off, wv
        self.idx = sym.export("IDX")
        self.relpos = sym.export("RELPOS")
        self.asm_ptr = sym.export("ASM_PTR")
        self.asm_col = sym.export("ASM_COL")
        self.asm_nz = sym.export("ASM_NZ")
        self.ea_ptr = sym.export("EA_PTR")
        self.ea_src = sym.export("EA_SRC")
        self.level_ptr = sym.export("LEVEL_PTR")
        self.level_fronts = sym.export("LEVEL_FRONTS")
        self.perm = sym.export("PERM")
        self.iperm = sym.export("IPERM")
        self.n = self.perm.size
        rows = int(self.fr[:, 1].sum())
        self.row_front = np.zeros(rows, dtype=np.int64)
        for t, (ns, f, row0, *_r) in enumerate(self.fr):
            self.row_front[row0:row0 + f] = t

    def levels(self, reverse=False):
        L = self.level_ptr.size - 1
        order = range(L - 1, -1, -1) if reverse else range(L)
        for l in order:
            yield self.level_fronts[self.level_ptr[l]:self.level_ptr[l + 1]]

    def factor(self, data):
        """data: CSC values (nnz,) complex.  Returns list of dense fronts."""
        F = [None] * len(self.fr)
        for lvl in self.levels():
            for t in lvl:
                ns, f, row0 = int(self.fr[t, 0]), int(self.fr[t, 1]), int(self.fr[t, 2])
                A = np.zeros((f, f), dtype=complex)
                for a in range(f):
                    r = row0 + a
                    for e in range(self.asm_ptr[r], self.asm_ptr[r + 1]):
                        A[a, self.asm_col[e]] += data[self.asm_nz[e]]
                    for e in range(self.ea_ptr[r], self.ea_ptr[r + 1]):
                        src = self.ea_src[e]
                        c = self.row_front[src]
                        cns, cf, crow0 = int(self.fr[c, 0]), int(self.fr[c, 1]), int(self.fr[c, 2])
                        lr = src - crow0
                        for b in range(cns, cf):
                            A[a, self.relpos[crow0 + b]] += F[c][lr, b]
                for k in range(ns):
                    A[k + 1:, k] /= A[k, k]
                    A[k + 1:, k + 1:] -= np.outer(A[k + 1:, k], A[k, k + 1:])
                F[t] = A
        return F

    def _gather(self, F, WV, t, rhs_perm):
        ns, f, row0 = int(self.fr[t, 0]), int(self.fr[t, 1]), int(self.fr[t, 2])
        w = np.zeros(f, dtype=complex)
        for a in range(f):
            r = row0 + a
            if a < ns:
                w[a] = rhs_perm[self.idx[r]]
            for e in range(self.ea_ptr[r], self.ea_ptr[r + 1]):
                w[a] += WV[self.ea_src[e]]
        return w

    def solve(self, F, b, transpose=False):
        """x = A^{-1} b (or A^{-T} b, non-conjugate), b in caller numbering."""
        bp = b[self.perm]
        WV = np.zeros(int(self.fr[:, 1].sum()), dtype=complex)
        Y = np.zeros(self.n, dtype=complex)
        X = np.zeros(self.n, dtype=complex)
        for lvl in self.levels():
            for t in lvl:
                ns, f, row0, col0 = (int(v) for v in self.fr[t, :4])
                w = self._gather(F, WV, t, bp)
                A = F[t]
                if not transpose:         # L (unit lower)
                    for k in range(ns):
                        w[k + 1:] -= A[k + 1:, k] * w[k]
                else:                     # U^T
                    for k in range(ns):
                        w[k] /= A[k, k]
                        w[k + 1:] -= A[k, k + 1:] * w[k]
                WV[row0:row0 + f] = w
                Y[col0:col0 + ns] = w[:ns]
        for lvl in self.levels(reverse=True):
            for t in lvl:
                ns, f, row0, col0 = (int(v) for v in self.fr[t, :4])
                A = F[t]
                xr = X[self.idx[row0 + ns:row0 + f]]
                if not transpose:         # U
                    v = Y[col0:col0 + ns] - A[:ns, ns:] @ xr
                    for k in range(ns - 1, -1, -1):
                        v[k] /= A[k, k]
                        v[:k] -= A[:k, k] * v[k]
                else:                     # L^T (unit upper)
                    v = Y[col0:col0 + ns] - A[ns:, :ns].T @ xr
                    for k in range(ns - 1, -1, -1):
                        v[:k] -= A[k, :k] * v[k]
                X[col0:col0 + ns] = v
        out = np.zeros(self.n, dtype=complex)
        out[self.perm] = X
        return out

    # ---------------------------------------------------------------- symmetric mode
    def solve_sym(self, F, b, sym, data, transpose=False):
        """Symmetric-mode solve (pfr_symbolic_options.symmetric = 1), as libpfr runs it:
        the factorisation is of the decoupled matrix (Dirichlet columns left out); the
        U solve uses U12 = diag(U11) L21^T (U12 never formed).  forward: Dirichlet columns
        moved to the right-hand side first; transpose: Dirichlet rows of the solution
        corrected after the solve (kernels.hip k_dirichlet_rhs / k_dirichlet_post)."""
        dirs = sym.export("DIRICHLET")
        cpl = sym.export("COUPLING")
        bp = b[self.perm].astype(complex)
        if not transpose:
            for p_i, ds, nz in cpl:
                p_d, nz_dd = dirs[ds]
                bp[p_i] -= data[nz] * bp[p_d] / data[nz_dd]
        WV = np.zeros(int(self.fr[:, 1].sum()), dtype=complex)
        Y = np.zeros(self.n, dtype=complex)
        X = np.zeros(self.n, dtype=complex)
        for lvl in self.levels():
            for t in lvl:
                ns, f, row0, col0 = (int(v) for v in self.fr[t, :4])
                w = self._gather(F, WV, t, bp)
                A = F[t]
                for k in range(ns):
                    w[k + 1:] -= A[k + 1:, k] * w[k]
                WV[row0:row0 + f] = w
                Y[col0:col0 + ns] = w[:ns]
        for lvl in self.levels(reverse=True):
            for t in lvl:
                ns, f, row0, col0 = (int(v) for v in self.fr[t, :4])
                A = F[t]
                xr = X[self.idx[row0 + ns:row0 + f]]
                U12 = np.diag(A)[:ns, None] * A[ns:, :ns].T
                v = Y[col0:col0 + ns] - U12 @ xr
                for k in range(ns - 1, -1, -1):
                    v[k] /= A[k, k]
                    v[:k] -= A[:k, k] * v[k]
                X[col0:col0 + ns] = v
        if transpose:
            for p_i, ds, nz in cpl:
                p_d, nz_dd = dirs[ds]
                X[p_d] -= data[nz] * X[p_i] / data[nz_dd]
        out = np.zeros(self.n, dtype=complex)
        out[self.perm] = X
        return out
