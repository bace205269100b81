"""Triangular meshes for the plate and for the accelerometer averaging disc.

The reference builds both meshes with FreeFEM++ ``buildmesh``
(``source/jax_plate/geometry/sh_i.edp:22-31`` for the strip,
``source/jax_plate/pyFFInterface.py:199-202`` for the disc ``accTh``).  FreeFEM
is not available here, so this module generates structured equivalents with
the same geometry and the same boundary labelling:

* strip ``[0, Lx] x [-Ly/2, Ly/2]``; the short side ``x = Lx`` carries label 1
  (clamped + kinematically excited, ``sh_i.edp:25``), every other side label 0;
* disc of radius ``0.3 * r_accel`` centred at the test point
  (``pyFFInterface.py:199-201``), sampled by concentric rings whose outer ring
  has 64 nodes like ``buildmesh(CAccin(64))``.

Meshes differ from FreeFEM's Delaunay meshes, so the reference's printed known
answers (``examples/cpu_benchmark.py:24``) are not reproducible bit-for-bit.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class TriMesh:
    """A conforming triangulation with an edge table.

    Attributes
    ----------
    vertices : (V, 2) float64
    triangles : (T, 3) int64, counter-clockwise
    edges : (E, 2) int64, each row sorted ascending (global orientation)
    tri_edges : (T, 3) int64, ``tri_edges[t, k]`` is the edge opposite local vertex k
    vertex_label1 : (V,) bool, vertex lies on a label-1 boundary edge
    edge_label1 : (E,) bool, edge is a label-1 boundary edge
    """

    vertices: np.ndarray
    triangles: np.ndarray
    edges: np.ndarray
    tri_edges: np.ndarray
    vertex_label1: np.ndarray
    edge_label1: np.ndarray

    @property
    def n_vertices(self) -> int:
        return self.vertices.shape[0]

    @property
    def n_edges(self) -> int:
        return self.edges.shape[0]

    @property
    def n_triangles(self) -> int:
        return self.triangles.shape[0]

    def areas(self) -> np.ndarray:
        p = self.vertices[self.triangles]
        d1 = p[:, 1] - p[:, 0]
        d2 = p[:, 2] - p[:, 0]
        return 0.5 * (d1[:, 0] * d2[:, 1] - d1[:, 1] * d2[:, 0])


def _build_edges(triangles: np.ndarray, n_vertices: int):
    loc = np.array([[1, 2], [2, 0], [0, 1]])
    pairs = triangles[:, loc]                      # (T, 3, 2)
    pairs = np.sort(pairs, axis=2)
    keys = pairs[:, :, 0] * n_vertices + pairs[:, :, 1]
    uniq, inv = np.unique(keys.ravel(), return_inverse=True)
    edges = np.stack([uniq // n_vertices, uniq % n_vertices], axis=1)
    return edges.astype(np.int64), inv.reshape(-1, 3).astype(np.int64)


def strip_mesh(length: float, width: float, nx: int, ny: int,
               clamp_tol: float = 1e-12) -> TriMesh:
    """Structured triangulation of ``[0, length] x [-width/2, width/2]``.

    Cells are split along alternating diagonals (checkerboard) so the mesh has
    no preferred direction.  The side ``x = length`` is label 1.
    """
    if nx < 1 or ny < 1:
        raise ValueError("nx and ny must be positive")
    xs = np.linspace(0.0, length, nx + 1)
    ys = np.linspace(-width / 2.0, width / 2.0, ny + 1)
    X, Y = np.meshgrid(xs, ys, indexing="ij")       # vertex (i, j) -> i*(ny+1)+j
    vertices = np.stack([X.ravel(), Y.ravel()], axis=1)

    def vid(i, j):
        return i * (ny + 1) + j

    I, J = np.meshgrid(np.arange(nx), np.arange(ny), indexing="ij")
    I = I.ravel()
    J = J.ravel()
    a = vid(I, J)
    b = vid(I + 1, J)
    c = vid(I + 1, J + 1)
    d = vid(I, J + 1)
    flip = ((I + J) % 2).astype(bool)
    # diagonal a-c for even cells, b-d for odd cells; all triangles CCW
    t1 = np.where(flip[:, None], np.stack([a, b, d], 1), np.stack([a, b, c], 1))
    t2 = np.where(flip[:, None], np.stack([b, c, d], 1), np.stack([a, c, d], 1))
    triangles = np.concatenate([t1, t2], axis=0).astype(np.int64)

    edges, tri_edges = _build_edges(triangles, vertices.shape[0])
    vertex_label1 = np.abs(vertices[:, 0] - length) <= clamp_tol * max(1.0, length)
    edge_label1 = vertex_label1[edges[:, 0]] & vertex_label1[edges[:, 1]]
    return TriMesh(vertices, triangles, edges, tri_edges, vertex_label1, edge_label1)


def disc_nodes(center: tuple[float, float], radius: float, n_boundary: int = 64) -> np.ndarray:
    """Nodes of a P1 mesh of a disc, as concentric rings.

    Stands in for the P1 nodes of ``accTh = buildmesh(CAccin(64))``
    (``pyFFInterface.py:199-202``): the outer ring has ``n_boundary`` nodes and
    inner rings keep roughly the same spacing, so the unweighted nodal mean
    used by the reference functional (``Problem.py:460-462``) samples the disc
    nearly uniformly.
    """
    h = 2.0 * np.pi * radius / n_boundary
    n_rings = max(1, int(round(radius / h)))
    pts = [np.array([[0.0, 0.0]])]
    for k in range(1, n_rings + 1):
        rk = radius * k / n_rings
        nk = max(3, int(round(n_boundary * k / n_rings)))
        t = 2.0 * np.pi * (np.arange(nk) + 0.5 * (k % 2)) / nk
        pts.append(np.stack([rk * np.cos(t), rk * np.sin(t)], axis=1))
    nodes = np.concatenate(pts, axis=0)
    return nodes + np.asarray(center, dtype=np.float64)[None, :]


def locate_points(mesh: TriMesh, points: np.ndarray, tol: float = 1e-12):
    """Return (triangle index, barycentric coordinates) for every point.

    A point on a shared edge is assigned to the lowest-index containing
    triangle.  Raises if a point lies outside the mesh.
    """
    p = mesh.vertices[mesh.triangles]                 # (T, 3, 2)
    x0 = p[:, 0]
    d1 = p[:, 1] - x0
    d2 = p[:, 2] - x0
    det = d1[:, 0] * d2[:, 1] - d1[:, 1] * d2[:, 0]
    tri = np.full(points.shape[0], -1, dtype=np.int64)
    bary = np.zeros((points.shape[0], 3))
    # bounding-box prefilter keeps this O(P * candidates)
    lo = p.min(axis=1) - tol
    hi = p.max(axis=1) + tol
    for k, q in enumerate(points):
        cand = np.nonzero((q[0] >= lo[:, 0]) & (q[0] <= hi[:, 0]) &
                          (q[1] >= lo[:, 1]) & (q[1] <= hi[:, 1]))[0]
        r = q[None, :] - x0[cand]
        l1 = (r[:, 0] * d2[cand, 1] - r[:, 1] * d2[cand, 0]) / det[cand]
        l2 = (d1[cand, 0] * r[:, 1] - d1[cand, 1] * r[:, 0]) / det[cand]
        l0 = 1.0 - l1 - l2
        ok = np.nonzero((l0 >= -1e-10) & (l1 >= -1e-10) & (l2 >= -1e-10))[0]
        if ok.size == 0:
            raise ValueError(f"point {q} is outside the mesh")
        j = ok[0]
        tri[k] = cand[j]
        bary[k] = (l0[j], l1[j], l2[j])
    return tri, bary
