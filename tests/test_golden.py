"""Pin the restatements against fixtures produced by the REFERENCE code itself
(tests/golden/make_golden.py): Material.py transforms and the
load_matrices_unsymm block layout."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import plate_oracle as orc
from plate_inverse_problem_amd.Material import get_material
from plate_inverse_problem_amd.fem import block_layout, plate_varfs, strip_mesh
from plate_inverse_problem_amd.fem.layout import MATRIX_NAMES

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _records():
    with open(os.path.join(GOLDEN, "material_abd.json")) as f:
        return json.load(f)


def _cplx(pairs):
    return np.array([complex(a, b) for a, b in pairs])


def _close(got, ref, scale):
    return np.max(np.abs(np.asarray(got) - ref)) <= 1e-13 * scale


@pytest.mark.parametrize("rec", _records(), ids=lambda r: f"{r['atype']}-h{r['h']}")
def test_material_transform_matches_reference(rec):
    """Product (torch) transforms == reference Material.py outputs."""
    m = get_material(1500.0, rec["atype"], **rec["kwargs"])
    assert list(m.get_parameters()) == rec["params"]
    assert m.is_mps == rec["is_mps"]
    A, B, D = m.get_ABD_transform(rec["h"])(torch.tensor(rec["theta"], dtype=torch.float64), 0.0)
    refA, refB, refD = _cplx(rec["A"]), _cplx(rec["B"]), _cplx(rec["D"])
    sA = np.max(np.abs(refA))
    assert _close(A.numpy(), refA, sA)
    assert _close(D.numpy(), refD, np.max(np.abs(refD)))
    assert _close(B.numpy(), refB, sA * rec["h"])


@pytest.mark.parametrize("rec", _records(), ids=lambda r: f"{r['atype']}-h{r['h']}")
def test_oracle_transform_matches_reference(rec):
    """Oracle (numpy) transforms == reference Material.py outputs."""
    angles = rec["kwargs"].get("angles")
    A, B, D = orc.abd_transform(rec["atype"], rec["h"], rec["theta"], angles)
    refA, refB, refD = _cplx(rec["A"]), _cplx(rec["B"]), _cplx(rec["D"])
    sA = np.max(np.abs(refA))
    assert _close(A, refA, sA)
    assert _close(D, refD, np.max(np.abs(refD)))
    assert _close(B, refB, sA * rec["h"])


def test_orthotropic_d22_quirk():
    """Reference quirk Material.py:475: D22 = D11 / (E2/E1)."""
    m = get_material(1500.0, "orthotropic", E1=120e9, E2=8e9, G12=5e9, nu12=0.3, beta=0.01)
    _, _, D = m.get_ABD_transform(2e-3)(torch.tensor(m.get_parameters()))
    assert abs((D[3] / D[0]).real - 15.0) < 1e-12


def _load_layout(case):
    g = np.load(os.path.join(GOLDEN, f"layout_{case}.npz"))
    return g


@pytest.mark.parametrize("case,nx,ny", [("tiny", 4, 2), ("small", 10, 3)])
def test_block_layout_bit_exact(case, nx, ny):
    """26 system matrices, incl. explicit zeros, == reference load_matrices_unsymm
    post-processing (pyFFInterface.py:279-509) on the same varf input."""
    g = _load_layout(case)
    Lx, Ly, r = 100e-3, 20e-3, 3.8e-3
    ff = plate_varfs(strip_mesh(Lx, Ly, nx, ny), (r, Ly / 2 - r), r)
    mats, rhs, Lh, Mh = block_layout(ff)
    assert (Lh, Mh) == (int(g["Lh"]), int(g["Mh"]))
    assert len(mats) == 26 == len(MATRIX_NAMES)
    for k, m in enumerate(mats):
        c = m.tocoo()
        got = sorted(zip(c.row.tolist(), c.col.tolist(), c.data.tolist()))
        ref = sorted(zip(g[f"mat{k}_row"].tolist(), g[f"mat{k}_col"].tolist(), g[f"mat{k}_data"].tolist()))
        assert got == ref, MATRIX_NAMES[k]
    assert np.array_equal(rhs, g["rhs"])


def test_varf_inputs_reproducible():
    """The golden's varf inputs were made by this build's assembler: regenerate bit-exactly."""
    g = _load_layout("tiny")
    Lx, Ly, r = 100e-3, 20e-3, 3.8e-3
    ff = plate_varfs(strip_mesh(Lx, Ly, 4, 2), (r, Ly / 2 - r), r)
    for name in ("Sxx", "Rxxy", "Txyxy", "M33Correction"):
        c = ff[name].tocoo()
        assert np.array_equal(c.data, g[f"in_{name}_data"])
