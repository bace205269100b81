"""FE matrix source: meshes, P1/Morley element properties, Dirichlet semantics."""
import numpy as np
import pytest

from plate_inverse_problem_amd.Geometry import dofs_for_density
from plate_inverse_problem_amd.fem import MorleyBasis, plate_varfs, strip_mesh
from plate_inverse_problem_amd.fem.layout import union_pattern
from plate_inverse_problem_amd.fem.mesh import disc_nodes, locate_points


@pytest.fixture(scope="module")
def mesh():
    return strip_mesh(100e-3, 20e-3, 10, 3)


def test_mesh_counts_and_labels(mesh):
    assert mesh.n_vertices == 11 * 4
    assert mesh.n_triangles == 2 * 10 * 3
    assert mesh.n_edges == 3 * 10 * 3 + 10 + 3
    assert np.all(mesh.areas() > 0)
    assert np.isclose(mesh.areas().sum(), 100e-3 * 20e-3)
    assert mesh.vertex_label1.sum() == 4 and mesh.edge_label1.sum() == 3
    assert np.allclose(mesh.vertices[mesh.vertex_label1, 0], 100e-3)


def test_dof_count_formula():
    for ny in (3, 6, 12, 25):
        nx = int(round(ny * 5))
        m = strip_mesh(100e-3, 20e-3, nx, ny)
        assert dofs_for_density(ny) == 3 * m.n_vertices + m.n_edges


def test_morley_dofs_are_kronecker(mesh):
    """Each local basis function has value/normal-derivative DOFs = delta."""
    mb = MorleyBasis(mesh)
    T = mesh.n_triangles
    p = mesh.vertices[mesh.triangles]
    for k in range(3):
        val, gx, gy = mb.eval(np.arange(T), p[:, k])
        e = np.zeros(6)
        e[k] = 1
        assert np.allclose(val, e, atol=1e-10)
    for k in range(3):
        mid = 0.5 * (p[:, (k + 1) % 3] + p[:, (k + 2) % 3])
        val, gx, gy = mb.eval(np.arange(T), mid)
        n = mb.edge_normal[mesh.tri_edges[:, k]]
        dn = gx * n[:, :1] + gy * n[:, 1:]
        scale = np.abs(dn).max()
        e = np.zeros(6)
        e[3 + k] = 1
        assert np.allclose(dn / scale * scale, e, atol=1e-8 * scale)


def test_morley_reproduces_quadratics(mesh):
    """Interpolating a quadratic by its DOFs gives exact second derivatives."""
    mb = MorleyBasis(mesh)
    V = mesh.n_vertices
    w = lambda x, y: 3 * x * x - 2 * x * y + 5 * y * y + x - y       # noqa: E731
    gw = lambda x, y: (6 * x - 2 * y + 1, -2 * x + 10 * y - 1)       # noqa: E731
    dofs = np.zeros(V + mesh.n_edges)
    dofs[:V] = w(mesh.vertices[:, 0], mesh.vertices[:, 1])
    mid = mesh.vertices[mesh.edges].mean(axis=1)
    gx, gy = gw(mid[:, 0], mid[:, 1])
    dofs[V:] = gx * mb.edge_normal[:, 0] + gy * mb.edge_normal[:, 1]
    loc = dofs[mb.dofmap]                                            # (T, 6)
    assert np.allclose((mb.dxx * loc).sum(1), 6.0)
    assert np.allclose((mb.dxy * loc).sum(1), -2.0)
    assert np.allclose((mb.dyy * loc).sum(1), 10.0)


def test_varf_structure(mesh):
    ff = plate_varfs(mesh, (3.8e-3, 10e-3 - 3.8e-3), 3.8e-3)
    V, E = mesh.n_vertices, mesh.n_edges
    assert ff["Rxxx"].shape == (V, V + E)
    assert ff["Txxxx"].shape == (V + E, V + E)
    # FreeFEM orientation: rows = test.  Syx = Sxy^T on the unconstrained forms
    assert abs(ff["SxyL"] - ff["SyxL"].T).max() < 1e-12
    dm = np.nonzero(ff["vmarkerMh"])[0]
    keep = np.setdiff1d(np.arange(V + E), dm)               # on() rows break the transpose identity
    T1, T2 = ff["Txxyy"].toarray()[np.ix_(keep, keep)], ff["Tyyxx"].toarray()[np.ix_(keep, keep)]
    assert np.abs(T1 - T2.T).max() <= 1e-12 * np.abs(T1).max()
    # stiffness annihilates constants (no on() rows): row sums of SxxL vanish
    assert np.allclose(ff["SxxL"] @ np.ones(V), 0.0, atol=1e-12)
    # mass integrates to the area
    M11 = ff["M11"].toarray()
    d = np.nonzero(ff["vmarkerLh"])[0]
    free = np.setdiff1d(np.arange(V), d)
    assert np.all(np.diag(M11)[d] == 1.0)
    assert ff["M11Correction"].sum() > 0
    # tgv = -1: unit Dirichlet rows
    for name in ("Sxx", "Txxxx", "M33I2"):
        A = ff[name].toarray()
        dd = np.nonzero(ff["vmarkerLh" if name == "Sxx" else "vmarkerMh"])[0]
        assert np.allclose(A[dd][:, dd], np.eye(dd.size))
        off = A[dd].copy()
        off[np.arange(dd.size), dd] = 0
        assert np.all(off == 0)
    # P1 weights and the Morley vertex-value functions are partitions of unity
    assert np.allclose(np.asarray(ff["interpL"].sum(1)), 1.0)
    assert np.allclose(ff["interp"].toarray()[:, :V].sum(1), 1.0)
    assert free.size > 0


def test_disc_and_location(mesh):
    nodes = disc_nodes((0.01, 0.0), 1e-3, 64)
    assert np.allclose(np.linalg.norm(nodes - [0.01, 0.0], axis=1).max(), 1e-3)
    tri, bary = locate_points(mesh, nodes)
    rec = np.einsum("pk,pkd->pd", bary, mesh.vertices[mesh.triangles[tri]])
    assert np.allclose(rec, nodes)


def test_union_pattern_csc_order(mesh):
    from plate_inverse_problem_amd.fem import block_layout
    ff = plate_varfs(mesh, (3.8e-3, 10e-3 - 3.8e-3), 3.8e-3)
    mats, rhs, Lh, Mh = block_layout(ff)
    up = union_pattern(mats)
    n = up.n
    keys = up.rows.astype(np.int64) + n * up.cols.astype(np.int64)
    assert np.all(np.diff(keys) > 0)                 # sorted (CSC order), unique
    assert np.array_equal(np.diff(up.colptr), np.bincount(up.cols, minlength=n))
    for k, m in enumerate(mats):                     # values scattered exactly
        assert np.allclose(up.values[k].sum(), m.sum())
