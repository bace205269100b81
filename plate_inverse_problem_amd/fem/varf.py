"""P1 (in-plane) + Morley (bending) variational forms for the laminated plate.

This is the build's replacement for the FreeFEM++ varf script that the
reference generates in ``source/jax_plate/pyFFInterface.py:175-275`` and runs
through ``pyFreeFem`` (``FreeFemIO.py:247-305``).  It produces a dict with the
SAME keys, shapes and orientation as the reference's ``ff_output``:

* every matrix is ``(n_test, n_trial)``: rows are the test function (``r`` or
  ``t``), columns the unknown (``u`` or ``w``), FreeFEM's convention -- e.g.
  ``Rxxx`` is ``Lh x Mh`` (``pyFFInterface.py:233-241`` then ``move(KB11, 2, 0)``
  at ``:403-404`` shifts its columns into the w block);
* varfs carrying ``+ on(1, ...)`` are assembled with ``tgv = -1``
  (``pyFFInterface.py:176``, ``pyFreeFem/functions.py:62-65``): every Dirichlet
  row becomes a unit row, the row's structural zeros are kept;
* ``vBCMh`` is 1 on clamped vertex DOFs (``w = funcBC = 1``) and 0 on clamped
  normal-derivative DOFs (``wx = wy = 0``), ``pyFFInterface.py:185-197``.

Spaces: ``Lh`` = P1 on vertices.  ``Mh`` = Morley: DOFs are the vertex values
(first ``V``) followed by the edge-midpoint normal derivatives (``E``), normal of
each global edge fixed by the sorted vertex pair.  Second derivatives of a
Morley function are constant per triangle, so the ``T****`` and ``R***`` forms
are exact; mass-type forms use the 7-point degree-5 Dunavant rule (exact for
the degree-4 ``M33`` integrand; the ``indAccel`` corrections are evaluated at
those points, as FreeFEM evaluates a ``func`` at quadrature points).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from .mesh import TriMesh, disc_nodes, locate_points

# Dunavant degree-5 rule on the reference triangle (barycentric, weights sum 1)
_A1, _B1, _W1 = 0.059715871789770, 0.470142064105115, 0.132394152788506
_A2, _B2, _W2 = 0.797426985353087, 0.101286507323456, 0.125939180544827
QUAD_BARY = np.array([
    [1 / 3, 1 / 3, 1 / 3],
    [_A1, _B1, _B1], [_B1, _A1, _B1], [_B1, _B1, _A1],
    [_A2, _B2, _B2], [_B2, _A2, _B2], [_B2, _B2, _A2],
])
QUAD_W = np.array([0.225, _W1, _W1, _W1, _W2, _W2, _W2])


class MorleyBasis:
    """Per-triangle Morley shape functions, vectorised over all triangles.

    Local DOFs 0..2: values at the triangle's vertices; 3..5: normal derivative
    (global edge normal) at the midpoint of the edge opposite local vertex k.
    """

    def __init__(self, mesh: TriMesh):
        self.mesh = mesh
        p = mesh.vertices[mesh.triangles]                      # (T, 3, 2)
        self.center = p.mean(axis=1)                           # (T, 2)
        e_len = np.linalg.norm(p[:, [1, 2, 0]] - p[:, [2, 0, 1]], axis=2)
        self.h = e_len.max(axis=1)                             # (T,)

        # global edge normals
        ev = mesh.vertices[mesh.edges]                         # (E, 2, 2)
        t = ev[:, 1] - ev[:, 0]
        n = np.stack([t[:, 1], -t[:, 0]], axis=1)
        self.edge_normal = n / np.linalg.norm(n, axis=1, keepdims=True)

        T = mesh.n_triangles
        D = np.zeros((T, 6, 6))
        for k in range(3):
            xi = (p[:, k] - self.center) / self.h[:, None]
            D[:, k] = self._mono(xi)
        for k in range(3):
            a, b = p[:, (k + 1) % 3], p[:, (k + 2) % 3]
            mid = 0.5 * (a + b)
            xi = (mid - self.center) / self.h[:, None]
            nrm = self.edge_normal[mesh.tri_edges[:, k]]       # (T, 2)
            gx, gy = self._dmono(xi)
            D[:, 3 + k] = (nrm[:, :1] * gx + nrm[:, 1:] * gy) / self.h[:, None]
        # D[k, m] = DOF k of monomial m; basis phi_j = sum_m C[m, j] mono_m with
        # DOF_k(phi_j) = delta_kj  ->  C = D^-1
        self.C = np.linalg.inv(D)
        hh = self.h[:, None] ** 2
        self.dxx = 2.0 * self.C[:, 3, :] / hh                  # (T, 6)
        self.dxy = self.C[:, 4, :] / hh
        self.dyy = 2.0 * self.C[:, 5, :] / hh

        V = mesh.n_vertices
        self.dofmap = np.concatenate([mesh.triangles, V + mesh.tri_edges], axis=1)

    @staticmethod
    def _mono(xi):
        x, y = xi[..., 0], xi[..., 1]
        one = np.ones_like(x)
        return np.stack([one, x, y, x * x, x * y, y * y], axis=-1)

    @staticmethod
    def _dmono(xi):
        x, y = xi[..., 0], xi[..., 1]
        z = np.zeros_like(x)
        o = np.ones_like(x)
        gx = np.stack([z, o, z, 2 * x, y, z], axis=-1)
        gy = np.stack([z, z, o, z, x, 2 * y], axis=-1)
        return gx, gy

    def eval(self, tri: np.ndarray, pts: np.ndarray):
        """Values and gradients of the 6 local basis functions of ``tri`` at ``pts``.

        ``tri``: (P,), ``pts``: (P, 2) -> (val (P,6), gx (P,6), gy (P,6)).
        """
        xi = (pts - self.center[tri]) / self.h[tri, None]
        C = self.C[tri]                                        # (P, 6, 6)
        val = np.einsum("pm,pmj->pj", self._mono(xi), C)
        gx, gy = self._dmono(xi)
        gx = np.einsum("pm,pmj->pj", gx, C) / self.h[tri, None]
        gy = np.einsum("pm,pmj->pj", gy, C) / self.h[tri, None]
        return val, gx, gy


def _p1_grads(mesh: TriMesh):
    p = mesh.vertices[mesh.triangles]
    area = mesh.areas()
    # grad lambda_k = rot(edge opposite k) / (2 area)
    e = p[:, [2, 0, 1]] - p[:, [1, 2, 0]]                      # edge opposite k: p[k+2]-p[k+1]
    gx = -e[:, :, 1] / (2 * area[:, None])
    gy = e[:, :, 0] / (2 * area[:, None])
    return gx, gy, area


def _assemble(rows_map, cols_map, elem, n_rows, n_cols):
    """Sum element matrices ``elem`` (T, a, b) into an (n_rows, n_cols) CSR matrix."""
    T, a, b = elem.shape
    r = np.repeat(rows_map[:, :, None], b, axis=2).ravel()
    c = np.repeat(cols_map[:, None, :], a, axis=1).ravel()
    m = sp.coo_matrix((elem.ravel(), (r, c)), shape=(n_rows, n_cols)).tocsr()
    m.sort_indices()
    return m


def _apply_on(mat: sp.csr_matrix, dofs: np.ndarray) -> sp.csr_matrix:
    """FreeFEM ``on(...)`` with ``tgv = -1``: unit Dirichlet rows, structure kept."""
    old = mat
    coo_old = old.tocoo()
    is_d = np.zeros(old.shape[0], dtype=bool)
    is_d[dofs] = True
    keep = ~is_d[coo_old.row]
    r = [coo_old.row[keep]]
    c = [coo_old.col[keep]]
    v = [coo_old.data[keep]]
    dr = coo_old.row[~keep]
    dc = coo_old.col[~keep]
    r.append(dr)
    c.append(dc)
    v.append(np.where(dr == dc, 1.0, 0.0))
    has_diag = np.zeros(old.shape[0], dtype=bool)
    has_diag[dr[dr == dc]] = True
    miss = dofs[~has_diag[dofs]]
    r.append(miss)
    c.append(miss)
    v.append(np.ones(miss.size))
    out = sp.csr_matrix((np.concatenate(v), (np.concatenate(r), np.concatenate(c))),
                        shape=old.shape)
    out.sort_indices()
    return out


def _indicator(x, y, xa, ya, ra, eps=1e-8):
    """``indAccel`` of ``sh_i.edp:34``."""
    return 0.5 * (1.0 + np.sign(ra ** 2 + eps - (x - xa) ** 2 - (y - ya) ** 2))


def plate_varfs(mesh: TriMesh, accel_xy: tuple[float, float], accel_r: float,
                inner_mult: float = 0.3, n_disc: int = 64) -> dict:
    """Assemble every varf/vector of ``pyFFInterface.py:175-275`` on ``mesh``.

    Returns a dict keyed like the reference's ``ff_output``.
    """
    V, E = mesh.n_vertices, mesh.n_edges
    Lh, Mh = V, V + E
    xa, ya = accel_xy

    gx, gy, area = _p1_grads(mesh)
    mb = MorleyBasis(mesh)
    tri_v = mesh.triangles
    dm = mb.dofmap

    # quadrature points
    P = mesh.vertices[mesh.triangles]
    qpts = np.einsum("qk,tkd->tqd", QUAD_BARY, P)             # (T, Q, 2)
    ind = _indicator(qpts[..., 0], qpts[..., 1], xa, ya, accel_r)  # (T, Q)
    wq = QUAD_W[None, :] * area[:, None]                        # (T, Q)

    # P1 values at quadrature points = barycentric coordinates
    lam = np.broadcast_to(QUAD_BARY[None], (mesh.n_triangles, 7, 3))
    # Morley values / gradients at quadrature points
    T = mesh.n_triangles
    tri_rep = np.repeat(np.arange(T), 7)
    mv, mgx, mgy = mb.eval(tri_rep, qpts.reshape(-1, 2))
    mv = mv.reshape(T, 7, 6)
    mgx = mgx.reshape(T, 7, 6)
    mgy = mgy.reshape(T, 7, 6)

    A = area[:, None, None]
    out = {}

    def outer(a, b):
        return a[:, :, None] * b[:, None, :]

    # --- Lh x Lh (rows test r, cols trial u) -------------------------------
    lh_elem = {
        "Sxx": A * outer(gx, gx),
        "Sxy": A * outer(gx, gy),     # dx(r) * dy(u)
        "Syx": A * outer(gy, gx),     # dx(u) * dy(r)
        "Syy": A * outer(gy, gy),
        "M11": np.einsum("tq,tqi,tqj->tij", wq, lam, lam),
        "M11Correction": np.einsum("tq,tqi,tqj->tij", wq * ind, lam, lam),
    }
    d_lh = np.nonzero(mesh.vertex_label1)[0]
    for name, el in lh_elem.items():
        m = _assemble(tri_v, tri_v, el, Lh, Lh)
        if name in ("Sxx", "Sxy", "Syx", "Syy"):
            out[name + "L"] = m.copy()
        out[name] = _apply_on(m, d_lh)

    # --- Lh x Mh (rows test r in Lh, cols trial w in Mh) --------------------
    lm_elem = {
        "Rxxx": A * outer(gx, mb.dxx), "Rxyy": A * outer(gx, mb.dyy),
        "Rxxy": A * outer(gx, mb.dxy), "Ryxx": A * outer(gy, mb.dxx),
        "Ryyy": A * outer(gy, mb.dyy), "Ryxy": A * outer(gy, mb.dxy),
    }
    for name, el in lm_elem.items():
        out[name] = _assemble(tri_v, dm, el, Lh, Mh)

    # --- Mh x Mh (rows test t, cols trial w) --------------------------------
    xx, xy, yy = mb.dxx, mb.dxy, mb.dyy
    mm_elem = {
        "Txxxx": A * outer(xx, xx),   # dxx(w) dxx(t): [i=test][j=trial]
        "Txxyy": A * outer(yy, xx),   # dxx(w) dyy(t)
        "Tyyxx": A * outer(xx, yy),   # dyy(w) dxx(t)
        "Txxxy": A * outer(xy, xx),   # dxx(w) dxy(t)
        "Txyxx": A * outer(xx, xy),   # dxy(w) dxx(t)
        "Txyyy": A * outer(yy, xy),   # dxy(w) dyy(t)
        "Tyyxy": A * outer(xy, yy),   # dyy(w) dxy(t)
        "Txyxy": A * outer(xy, xy),
        "Tyyyy": A * outer(yy, yy),
        "M33": np.einsum("tq,tqi,tqj->tij", wq, mv, mv),
        "M33Correction": np.einsum("tq,tqi,tqj->tij", wq * ind, mv, mv),
        "M33I2": np.einsum("tq,tqi,tqj->tij", wq, mgx, mgx) + np.einsum("tq,tqi,tqj->tij", wq, mgy, mgy),
        "M33I2Correction": np.einsum("tq,tqi,tqj->tij", wq * ind, mgx, mgx)
        + np.einsum("tq,tqi,tqj->tij", wq * ind, mgy, mgy),
    }
    d_mh_v = np.nonzero(mesh.vertex_label1)[0]
    d_mh_e = V + np.nonzero(mesh.edge_label1)[0]
    d_mh = np.concatenate([d_mh_v, d_mh_e])
    for name, el in mm_elem.items():
        out[name] = _apply_on(_assemble(dm, dm, el, Mh, Mh), d_mh)

    # --- Dirichlet vectors ---------------------------------------------------
    out["vBCLh"] = np.zeros(Lh)
    vbc = np.zeros(Mh)
    vbc[d_mh_v] = 1.0                          # w = funcBC = 1; wx = wy = 0 -> 0
    out["vBCMh"] = vbc
    mk_l = np.zeros(Lh)
    mk_l[d_lh] = 1.0
    out["vmarkerLh"] = mk_l
    mk_m = np.zeros(Mh)
    mk_m[d_mh_v] = 100.0
    en = mb.edge_normal[d_mh_e - V]
    mk_m[d_mh_e] = 200.0 * en[:, 0] + 300.0 * en[:, 1]
    out["vmarkerMh"] = mk_m

    # --- interpolation onto the averaging disc (pyFFInterface.py:199-212) ----
    nodes = disc_nodes((xa, ya), inner_mult * accel_r, n_disc)
    tri, bary = locate_points(mesh, nodes)
    Pn = nodes.shape[0]
    rows = np.repeat(np.arange(Pn), 3)
    out["interpL"] = sp.csr_matrix((bary.ravel(), (rows, mesh.triangles[tri].ravel())), shape=(Pn, Lh))
    val, dvx, dvy = mb.eval(tri, nodes)
    rows6 = np.repeat(np.arange(Pn), 6)
    cols6 = dm[tri].ravel()
    out["interp"] = sp.csr_matrix((val.ravel(), (rows6, cols6)), shape=(Pn, Mh))
    out["interpWx"] = sp.csr_matrix((dvx.ravel(), (rows6, cols6)), shape=(Pn, Mh))
    out["interpWy"] = sp.csr_matrix((dvy.ravel(), (rows6, cols6)), shape=(Pn, Mh))
    out["xtest"] = float(xa)
    out["ytest"] = float(ya)
    out["tgv"] = -1.0
    out["Th"] = mesh
    return out
