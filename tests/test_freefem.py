"""FreeFEM-exported matrices (fem.freefem): the reader against the reference's own parsers.

``tests/golden/freefem_stream.npz`` (tests/golden/make_golden.py, ``make_freefem_golden``) holds a
FreeFem++-format stdout stream of every output the reference's matrix-export script prints
(``pyFFInterface.py:175-275``; FreeFem++ 4.x and 3.x matrix formats), the same outputs parsed by
the REFERENCE pyFreeFem (``FreeFem_str_to_matrix`` / ``_to_vector`` / ``_to_mesh``), and the
reference ``load_matrices_unsymm`` layout of the parsed dict.  Bit-exact agreement is required.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

from plate_inverse_problem_amd.fem import freefem as ffio
from plate_inverse_problem_amd.fem.layout import load_matrices_unsymm

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "freefem_stream.npz"))


def _coo(prefix, shape=None):
    r, c, d = G[prefix + "_row"], G[prefix + "_col"], G[prefix + "_data"]
    shape = tuple(G[prefix + "_shape"]) if shape is None else shape
    return sp.csr_matrix((d, (r, c)), shape=shape)


def _same(a, b):
    a, b = sp.csr_matrix(a), sp.csr_matrix(b)
    a.sum_duplicates()
    b.sum_duplicates()
    a.sort_indices()
    b.sort_indices()
    return (a.shape == b.shape and np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
            and np.array_equal(a.data, b.data))


@pytest.mark.parametrize("version", [4, 3])
def test_reader_matches_reference_parsers(version):
    text = G[f"stream_v{version}"].tobytes().decode()
    out = ffio.parse_output(text)
    for name, kind in ffio.PLATE_OUTPUTS.items():
        ref = f"v{version}_{name}"
        if kind == "matrix":
            assert _same(out[name], _coo(ref)), name
        elif kind == "mesh":
            m = out[name]
            assert np.array_equal(m.vertices[:, 0], G[ref + "_x"]) and np.array_equal(m.vertices[:, 1], G[ref + "_y"])
            assert np.array_equal(m.triangles, G[ref + "_triangles"])
        else:
            assert np.array_equal(np.atleast_1d(np.asarray(out[name], dtype=np.float64)), np.atleast_1d(G[ref])), name


def test_layout_of_freefem_output_matches_reference():
    ff = ffio.load_freefem_output(G["stream_v4"].tobytes().decode())
    mats, rhs, interp, interpL, Lh, Mh, _, interpWx, interpWy = load_matrices_unsymm(ff)
    n = 2 * Lh + Mh
    for k, m in enumerate(mats):
        ref = sp.csr_matrix((G[f"layout_mat{k}_data"], (G[f"layout_mat{k}_row"], G[f"layout_mat{k}_col"])),
                            shape=(n, n))
        c = m.tocoo()
        assert np.array_equal(c.row, G[f"layout_mat{k}_row"]) and np.array_equal(c.col, G[f"layout_mat{k}_col"])
        assert np.array_equal(c.data, G[f"layout_mat{k}_data"]), k
        assert _same(m, ref)
    assert np.array_equal(rhs, G["layout_rhs"])
    for key, v in (("interp", interp), ("interpL", interpL), ("interpWx", interpWx), ("interpWy", interpWy)):
        assert np.array_equal(np.asarray(v), G[f"layout_{key}"]), key


def test_round_trip_and_problem_from_freefem_output():
    """This build's varfs -> FreeFEM stream -> reader: identical matrices, and a Problem built from the
    stream has the same union pattern and values as one built from the native mesh."""
    from plate_inverse_problem_amd.fem import strip_mesh, plate_varfs
    from helpers import make_geometry, make_material
    from plate_inverse_problem_amd.Geometry import Geometry
    from plate_inverse_problem_amd.Problem import Problem
    geom, acc = make_geometry(ny=3)
    mesh = strip_mesh(geom.length, geom.width, geom.nx, geom.ny)
    ff = plate_varfs(mesh, (geom.accel_x, geom.accel_y), geom.accel_r)
    ff["xtest"], ff["ytest"], ff["tgv"] = geom.accel_x, geom.accel_y, -1.0
    text = ffio.format_plate_output(ff, ffio.to_freefem_mesh(mesh))
    back = ffio.load_freefem_output(text)
    for name in ffio.PLATE_VARFS + ("interp", "interpL", "interpWx", "interpWy"):
        assert _same(back[name], ff[name]), name
    g2 = Geometry.from_freefem_output(text, height=geom.height, accelerometer=acc)
    assert g2.n_dofs == geom.n_dofs and g2.accel_x == geom.accel_x
    p1 = Problem(geom, make_material("orthotropic"), acc)
    p2 = Problem(g2, make_material("orthotropic"), acc)
    assert np.array_equal(p1.rows, p2.rows) and np.array_equal(p1.cols, p2.cols)
    assert np.array_equal(p1.mats, p2.mats) and np.array_equal(p1.vec, p2.vec)
    assert np.array_equal(p1.averaging_vectors(), p2.averaging_vectors())


def test_malformed_streams_raise():
    with pytest.raises(ffio.FreeFemFormatError):
        ffio.parse_output("nothing here")
    bad = ffio.format_output("Sxx", "# comment\n2 2 0  3\n1 1 1.0\n2 2 2.0\n")      # 3 coefficients announced
    with pytest.raises(ffio.FreeFemFormatError):
        ffio.parse_output(bad, {"Sxx": "matrix"})
