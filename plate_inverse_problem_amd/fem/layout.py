"""The 26-matrix block layout of the unsymmetric plate system and its CSC union.

Restates ``source/jax_plate/pyFFInterface.py:279-509`` (block layout of the
varf matrices into the ``N x N`` system, ``N = 2 Lh + Mh``) and
``source/jax_plate/Problem.py:313-345`` (union sparsity pattern in CSC order,
values of the 26 matrices scattered onto it).

The reference spells every block out by hand; here the layout is a table.
Each system matrix is a sum of *terms*; a term is

    (linear combination of varf matrices, (col_block, row_block),
     symmetrise?, rows to clear)

evaluated with the same scipy operations in the same order as the reference
(``resize`` -> ``move`` -> ``transp`` -> ``rmrows``; sums of sparse matrices
prune zero results exactly like the reference's ``+``), so the union pattern,
including the explicit zeros the reference carries, is reproduced.  Parity is
pinned by ``tests/golden/layout_*.npz`` (produced by running the reference's
own ``load_matrices_unsymm`` post-processing on the same varf input).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

# clear-rows keys: 'u' -> Dirichlet Lh rows (u block), 'v' -> same + Lh (v block),
# 'w' -> Dirichlet Mh rows + 2 Lh (w block).  pyFFInterface.py:346-358.
_U, _V, _W = "u", "v", "w"

# (name, [terms]); term = (((coef, varf), ...), (col_block, row_block), symmetrise, clear)
# Order of terms inside a matrix follows the reference's sums (floating-point
# association matters for 3-term sums).
LAYOUT = (
    ("KA11", [(((1, "Sxx"),), (0, 0), False, ())]),                           # :364
    ("KA12", [(((1, "SxyL"),), (1, 0), True, (_U, _V))]),                       # :369-373
    ("KA16", [(((1, "Sxy"), (1, "Syx")), (0, 0), False, ()),                    # :375-381
              (((1, "SxxL"),), (1, 0), True, (_U, _V))]),
    ("KA22", [(((1, "Syy"),), (1, 1), False, ())]),                             # :366-367
    ("KA26", [(((1, "SyyL"),), (1, 0), True, (_U, _V)),                         # :383-390
              (((1, "Sxy"), (1, "Syx")), (1, 1), False, ())]),
    ("KA66", [(((1, "Syy"),), (0, 0), False, ()),                               # :392-400
              (((1, "SyxL"),), (1, 0), True, (_U, _V)),
              (((1, "Sxx"),), (1, 1), False, ())]),
    ("KB11", [(((-1, "Rxxx"),), (2, 0), True, (_U, _W))]),                      # :403-407
    ("KB12", [(((-1, "Rxyy"),), (2, 0), True, (_U, _W)),                        # :415-425
              (((-1, "Ryxx"),), (2, 1), True, (_V, _W))]),
    ("KB16", [(((-1, "Ryxx"),), (2, 0), True, (_U, _W)),                        # :427-437
              (((-1, "Rxxx"),), (2, 1), True, (_V, _W))]),
    ("KB22", [(((-1, "Ryyy"),), (2, 1), True, (_V, _W))]),                      # :409-413
    ("KB26", [(((-2, "Rxxy"), (-1, "Ryyy")), (2, 0), True, (_U, _W)),           # :439-449
              (((-1, "Rxyy"), (-2, "Ryxy")), (2, 1), True, (_V, _W))]),
    ("KB66", [(((-2, "Ryxy"),), (2, 0), True, (_U, _W)),                        # :451-461
              (((-2, "Rxxy"),), (2, 1), True, (_V, _W))]),
    ("KD11", [(((1, "Txxxx"),), (2, 2), False, ())]),                           # :464-465
    ("KD12", [(((1, "Txxyy"), (1, "Tyyxx")), (2, 2), False, ())]),              # :467-468
    ("KD16", [(((1, "Txxxy"), (1, "Txyxx")), (2, 2), False, (), 2.0)]),         # :470-471  2*(...)
    ("KD22", [(((1, "Tyyyy"),), (2, 2), False, ())]),                           # :479-480
    ("KD26", [(((1, "Txyyy"), (1, "Tyyxy")), (2, 2), False, (), 2.0)]),         # :473-474  2*(...)
    ("KD66", [(((4, "Txyxy"),), (2, 2), False, ())]),                           # :476-477
    ("KM11", [(((1, "M11"),), (0, 0), False, ())]),                             # :483
    ("KM11Corr", [(((1, "M11Correction"),), (0, 0), False, ())]),               # :484
    ("KM22", [(((1, "M11"),), (1, 1), False, ())]),                             # :486-487
    ("KM22Corr", [(((1, "M11Correction"),), (1, 1), False, ())]),               # :488-489
    ("KM33", [(((1, "M33"),), (2, 2), False, ())]),                             # :491-492
    ("KM33Corr", [(((1, "M33Correction"),), (2, 2), False, ())]),               # :493-494
    ("KM33I2", [(((1, "M33I2"),), (2, 2), False, ())]),                         # :495-496
    ("KM33I2Corr", [(((1, "M33I2Correction"),), (2, 2), False, ())]),           # :497-498
)

MATRIX_NAMES = tuple(name for name, _ in LAYOUT)
assert len(MATRIX_NAMES) == 26


def _combine(ff: dict, combo, post_scale: float | None):
    out = None
    for coef, name in combo:
        m = ff[name]
        t = m if coef == 1 else coef * m
        out = t if out is None else out + t
    if post_scale is not None:
        out = post_scale * out
    return out


def block_layout(ff: dict):
    """Build the 26 system matrices from a varf dict (keys of ``plate_varfs``).

    Returns ``(mats, rhs_vec, Lh, Mh)``; ``mats`` are scipy sparse matrices in
    the reference's return order (``pyFFInterface.py:503-507``).
    """
    Lh = int(np.asarray(ff["vBCLh"]).size)
    Mh = int(np.asarray(ff["vBCMh"]).size)
    n = 2 * Lh + Mh
    d_lh = np.nonzero(np.asarray(ff["vmarkerLh"]))[0]
    d_mh = np.nonzero(np.asarray(ff["vmarkerMh"]))[0]
    clear_rows = {_U: d_lh, _V: d_lh + Lh, _W: d_mh + 2 * Lh}

    mats = []
    for name, terms in LAYOUT:
        total = None
        for term in terms:
            combo, (cb, rb), symm, clear = term[:4]
            post = term[4] if len(term) > 4 else None
            m = _combine(ff, combo, post).copy().tocoo()
            m.resize((n, n))
            m.col += cb * Lh
            m.row += rb * Lh
            if symm:
                m = (m + m.transpose(copy=True)).tocoo()
            for key in clear:
                hit = np.isin(m.row, clear_rows[key])
                m.data[hit] = 0
            total = m if total is None else total + m
        mats.append(total)

    rhs = np.zeros(n, dtype=np.float64)
    rhs[2 * Lh:] = np.asarray(ff["vBCMh"], dtype=np.float64)      # :500-501
    return mats, rhs, Lh, Mh


def load_matrices_unsymm(ff: dict):
    """Same return tuple as the reference ``load_matrices_unsymm`` (``:503-509``)."""
    mats, rhs, Lh, Mh = block_layout(ff)
    dense = {k: np.asarray(ff[k].todense()) for k in ("interp", "interpWx", "interpWy", "interpL")}
    return (mats, rhs, dense["interp"], dense["interpL"], Lh, Mh,
            ff["Th"], dense["interpWx"], dense["interpWy"])


@dataclass
class UnionPattern:
    """The CSC union pattern of the 26 matrices (``Problem.py:317-345``).

    ``values[k]`` holds matrix k on the pattern (zeros where it has no entry).
    ``rows``/``cols`` are the COO coordinates in CSC order (column-major,
    rows ascending within a column) -- the order the reference's solver state
    receives (``Sparse.py:100-116``).
    """

    n: int
    colptr: np.ndarray      # (n+1,) int32
    rowind: np.ndarray      # (nnz,) int32
    rows: np.ndarray        # (nnz,) int32
    cols: np.ndarray        # (nnz,) int32
    values: np.ndarray      # (26, nnz) float64

    @property
    def nnz(self) -> int:
        return int(self.rowind.size)


def union_pattern(mats) -> UnionPattern:
    n = mats[0].shape[0]
    coos = [m.tocoo() for m in mats]
    keys = np.array([], dtype=np.int64)
    for m in coos:
        keys = np.union1d(keys, m.row.astype(np.int64) + n * m.col.astype(np.int64))
    rows = (keys % n).astype(np.int32)
    cols = (keys // n).astype(np.int32)
    values = np.zeros((len(coos), keys.size), dtype=np.float64)
    for k, m in enumerate(coos):
        mk = m.row.astype(np.int64) + n * m.col.astype(np.int64)
        pos = np.searchsorted(keys, mk)
        np.add.at(values[k], pos, m.data)
    colptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(colptr, cols.astype(np.int64) + 1, 1)
    colptr = np.cumsum(colptr).astype(np.int32)
    return UnionPattern(n=n, colptr=colptr, rowind=rows.copy(), rows=rows, cols=cols, values=values)
