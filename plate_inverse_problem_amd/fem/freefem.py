"""FreeFEM++ text output: reader (and writer) for the exported varf matrices.

The reference builds the plate's FE matrices by running FreeFem++ on the geometry's ``.edp``
script followed by the varf block of ``source/jax_plate/pyFFInterface.py:175-275``, and parses
the program's standard output with the vendored pyFreeFem (``pyFreeFem/edpScript.py:67-82``,
``pyFreeFem/FreeFemIO.py:42-44, 56-133``).  FreeFem++ is not installed here, but a user who has
run that script elsewhere holds the text stream; this module turns it into the varf dict that
``fem.layout.load_matrices_unsymm`` lays out (``Geometry.from_freefem_output`` /
``Problem`` then take it from there), so FreeFEM-exported meshes reach the GPU solver.

Stream format (pyFreeFem conventions, restated):

* every output sits between two identical flag lines ``# FLAG > NAME`` (the name upper-cased,
  runs of non-alphanumerics and underscores turned into single spaces,
  ``FreeFemTools/edpTools.py:36-64``);
* matrix: FreeFem++'s ``cout << M`` -- a few comment lines, then a header of integers: FreeFem++
  3.x ``n m is_symmetric nnz`` with 1-based ``i j a_ij`` lines, FreeFem++ 4.x ``n m nnz`` + 4 more
  integers with 0-based lines (``FreeFemIO.py:70-97``); duplicate coordinates add up
  (``csr_matrix`` construction);
* array / vector: one value per line; real / int: one number;
* mesh: three flagged sub-blocks ``NODES`` (x y label), ``TRIANGLES`` (3 vertex ids, label),
  ``BOUNDARIES`` (2 vertex ids, label) (``FreeFemStatics.py:59-80``, ``FreeFemIO.py:117-133``).

Pinned against the reference parser itself (``FreeFem_str_to_matrix`` and the whole
``load_matrices_unsymm`` post-processing on a FreeFEM-format stream): ``tests/golden/freefem_*``.
"""
from __future__ import annotations

import io
import os
import re
import unicodedata
from dataclasses import dataclass

import numpy as np
import scipy.sparse as sp

# The outputs the reference script prints (pyFFInterface.py:217-275): name -> type
PLATE_VARFS = ("Sxx", "Sxy", "Syx", "Syy", "SxxL", "SxyL", "SyxL", "SyyL", "M11", "M11Correction",
               "Rxxx", "Rxyy", "Rxxy", "Ryxx", "Ryyy", "Ryxy",
               "Txxxx", "Txxyy", "Tyyxx", "Txxxy", "Txyxx", "Txyyy", "Tyyxy", "Txyxy", "Tyyyy",
               "M33", "M33Correction", "M33I2", "M33I2Correction")
PLATE_OUTPUTS = {**{k: "matrix" for k in PLATE_VARFS},
                 "vBCLh": "array", "vBCMh": "array", "vmarkerLh": "array", "vmarkerMh": "array",
                 "interp": "matrix", "interpWx": "matrix", "interpWy": "matrix", "interpL": "matrix",
                 "xtest": "real", "ytest": "real", "tgv": "real", "Th": "mesh"}


class FreeFemFormatError(ValueError):
    pass


def flag(name: str) -> str:
    """Flag line of an output (``flagize`` / ``FreeFemize(name, 'header')``)."""
    s = unicodedata.normalize("NFKD", name).encode("ASCII", "ignore").decode("utf8")
    s = re.sub(r"\W+", "_", s)
    return "# FLAG > " + " ".join(s.replace("_", " ").split()).upper()


def block(stream: str, name: str) -> str:
    """Text between the first two flag lines of ``name``."""
    f = flag(name) + "\n"
    parts = stream.split(f)
    if len(parts) < 3:
        raise FreeFemFormatError(f"output {name!r} ({f.strip()!r}) not found in the FreeFEM stream")
    return parts[1]


def parse_matrix(text: str, max_header_length: int = 15) -> sp.csr_matrix:
    """A FreeFem++ sparse matrix (3.x or 4.x text format) -> ``csr_matrix``."""
    lines = text.split("\n")
    header = None
    for i, line in enumerate(lines[:max_header_length]):
        try:
            nums = [int(w) for w in line.split()]
        except ValueError:
            continue
        if len(nums) >= 2:
            header, start = nums, i + 1
            break
    if header is None:
        raise FreeFemFormatError("no matrix header line (two or more integers) found")
    if len(header) == 4:                   # FreeFem++ 3.x: n m is_symmetric nnz, 1-based
        n, m, _, nnz = header
        base = 1
    elif len(header) == 7:                 # FreeFem++ 4.x: n m nnz + 4 integers, 0-based
        n, m, nnz = header[:3]
        base = 0
    else:
        raise FreeFemFormatError(f"unrecognised matrix header {header}")
    body = "\n".join(lines[start:start + nnz])
    vals = np.loadtxt(io.StringIO(body), dtype=np.float64, ndmin=2) if nnz > 0 else np.zeros((0, 3))
    if vals.shape != (nnz, 3):
        raise FreeFemFormatError(f"expected {nnz} 'i j a_ij' lines, got an array of shape {vals.shape}")
    i = vals[:, 0].astype(np.int64) - base
    j = vals[:, 1].astype(np.int64) - base
    return sp.csr_matrix((vals[:, 2], (i, j)), shape=(n, m))


def parse_vector(text: str) -> np.ndarray:
    """One value per line -> float64 array."""
    t = text.strip()
    return np.loadtxt(io.StringIO(t), dtype=np.float64, ndmin=1) if t else np.zeros(0)


@dataclass
class FreeFemMesh:
    """A FreeFem++ triangulation as exported by ``export_mesh_edp`` (0-based vertex ids)."""
    vertices: np.ndarray          # (nv, 2)
    node_labels: np.ndarray       # (nv,)
    triangles: np.ndarray         # (nt, 3)
    triangle_labels: np.ndarray   # (nt,)
    boundaries: np.ndarray        # (ne, 3): vertex, vertex, label


def parse_mesh(text: str) -> FreeFemMesh:
    t = "\n" + text + "\n"

    def part(key, dtype):
        f = "\n" + flag(key) + "\n"
        pieces = t.split(f)
        if len(pieces) < 3:
            raise FreeFemFormatError(f"mesh part {key!r} missing")
        body = pieces[1].strip()
        return np.loadtxt(io.StringIO(body), dtype=dtype, ndmin=2) if body else np.zeros((0, 3), dtype)

    nodes = part("nodes", np.float64)
    tri = part("triangles", np.int64)
    bnd = part("boundaries", np.int64)
    return FreeFemMesh(vertices=nodes[:, :2], node_labels=nodes[:, 2].astype(np.int64), triangles=tri[:, :3],
                       triangle_labels=tri[:, 3], boundaries=bnd)


_PARSERS = {"matrix": parse_matrix, "array": parse_vector, "vector": parse_vector,
            "real": lambda s: float(s), "int": lambda s: int(s), "mesh": parse_mesh}


def parse_output(stream: str, outputs: dict | None = None) -> dict:
    """Parse the named outputs (name -> 'matrix' | 'array' | 'vector' | 'real' | 'int' | 'mesh') of a
    FreeFem++ stdout stream; default: everything the plate script prints (``PLATE_OUTPUTS``)."""
    outputs = PLATE_OUTPUTS if outputs is None else outputs
    out = {}
    for name, kind in outputs.items():
        if kind not in _PARSERS:
            raise ValueError(f"unknown output type {kind!r}")
        out[name] = _PARSERS[kind](block(stream, name))
    return out


def load_freefem_output(source) -> dict:
    """The plate script's FreeFEM output (a path or the text itself) -> the varf dict
    ``fem.layout.load_matrices_unsymm`` expects (same keys as ``fem.varf.plate_varfs``)."""
    if isinstance(source, (str, os.PathLike)) and os.path.exists(source):
        with open(source) as f:
            text = f.read()
    elif isinstance(source, str):
        text = source
    else:
        raise TypeError("source must be a path or the FreeFEM output text")
    ff = parse_output(text)
    for k in ("vBCLh", "vBCMh", "vmarkerLh", "vmarkerMh"):
        ff[k] = np.asarray(ff[k], dtype=np.float64)
    return ff


# ----------------------------------------------------------------------------- writer
def _num(v) -> str:
    """Shortest round-trip decimal of a double."""
    return repr(float(v))


def format_matrix(M, version: int = 4) -> str:
    """``cout << M`` of FreeFem++ (``version`` 3: 1-based with the symmetric flag, 4: 0-based)."""
    c = sp.coo_matrix(M)
    n, m = c.shape
    buf = io.StringIO()
    if version == 3:
        buf.write("# Sparse Matrix (Morse)\n# first line: n m (is symmetic) nbcoef\n"
                  "# after for each nonzero coef:   i j a_ij where (i,j) \\in  {1,...,n}x{1,...,m} \n")
        buf.write(f"{n} {m} 0  {c.nnz}\n")
        base = 1
    else:
        buf.write("#  HashMatrix Matrix (COO) 0x0\n#    n       m        nnz     half     fortran   state  \n")
        buf.write(f"{n} {m} {c.nnz} 0 0 0 0\n")
        base = 0
    for i, j, v in zip(c.row, c.col, c.data):
        buf.write(f"{i + base:10d} {j + base:10d} {_num(v)}\n")
    return buf.getvalue()


def format_output(name: str, body: str) -> str:
    f = flag(name)
    return f"{f}\n{body if body.endswith(chr(10)) else body + chr(10)}{f}\n"


def format_mesh(vertices, node_labels, triangles, triangle_labels, boundaries) -> str:
    nodes = "".join(f"{_num(x)} {_num(y)} {int(lab)}\n" for (x, y), lab in zip(np.asarray(vertices), node_labels))
    tris = "".join(f"{a} {b} {c} {int(lab)}\n" for (a, b, c), lab in zip(np.asarray(triangles), triangle_labels))
    bnds = "".join(f"{a} {b} {int(lab)}\n" for a, b, lab in np.asarray(boundaries))
    return format_output("nodes", nodes) + "\n" + format_output("triangles", tris) + "\n" + \
        format_output("boundaries", bnds)


def format_plate_output(ff: dict, mesh: FreeFemMesh | None = None, version: int = 4) -> str:
    """A FreeFem++-style stream of the plate script's outputs from a varf dict (tests, and a
    way to hand this build's own discretisation to tools that read FreeFEM streams)."""
    parts = []
    for name, kind in PLATE_OUTPUTS.items():
        if kind == "matrix":
            body = format_matrix(ff[name], version)
        elif kind == "array":
            body = "".join(f"{_num(v)}\n" for v in np.asarray(ff[name], dtype=np.float64))
        elif kind == "real":
            body = f"{_num(ff.get(name, 0.0))}\n"
        else:
            m = mesh if mesh is not None else ff.get(name)
            if not isinstance(m, FreeFemMesh):
                raise ValueError("format_plate_output needs the mesh as a FreeFemMesh")
            body = format_mesh(m.vertices, m.node_labels, m.triangles, m.triangle_labels, m.boundaries)
        parts.append(format_output(name, body))
    return "".join(parts)


def to_freefem_mesh(mesh) -> FreeFemMesh:
    """This build's ``fem.mesh.TriMesh`` as a FreeFEM mesh: boundary edges (edges of one triangle)
    labelled 1 on the clamped side, 2 elsewhere; vertices labelled like their boundary edges."""
    tri_edges = np.asarray(mesh.tri_edges)
    count = np.bincount(tri_edges.ravel(), minlength=mesh.n_edges)
    bnd = np.nonzero(count == 1)[0]
    labels = np.where(np.asarray(mesh.edge_label1)[bnd], 1, 2)
    node_labels = np.zeros(mesh.n_vertices, dtype=np.int64)
    node_labels[np.asarray(mesh.edges)[bnd].ravel()] = np.repeat(labels, 2)
    node_labels[np.asarray(mesh.vertex_label1)] = 1
    boundaries = np.column_stack([np.asarray(mesh.edges)[bnd], labels]).astype(np.int64)
    return FreeFemMesh(vertices=np.asarray(mesh.vertices, dtype=np.float64), node_labels=node_labels,
                       triangles=np.asarray(mesh.triangles, dtype=np.int64),
                       triangle_labels=np.zeros(mesh.n_triangles, dtype=np.int64), boundaries=boundaries)
