"""Shared test helpers: canonical problems and the matching CPU oracle."""
from __future__ import annotations

import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

from plate_inverse_problem_amd.Accelerometer import Accelerometer  # noqa: E402
from plate_inverse_problem_amd.Geometry import Geometry, GeometryParams  # noqa: E402
from plate_inverse_problem_amd.Material import get_material  # noqa: E402

MATERIALS = {
    # cpu_benchmark.py:8-9 steel strip
    "isotropic": (7920.0, dict(E=200e9, G=75e9, beta=0.003)),
    # BASELINE.md C3 CFRP-like
    "orthotropic": (1500.0, dict(E1=120e9, E2=8e9, G12=5e9, nu12=0.3, beta=0.01)),
    "orthotropic_d4": (1500.0, dict(E1=120e9, E2=8e9, G12=5e9, nu12=0.3, b1=0.01, b2=0.02, b3=0.015, b4=0.005)),
    "sol": (1500.0, dict(E1=120e9, E2=8e9, G12=5e9, nu12=0.3, beta=0.01, angles=(0.0, 90.0))),   # B != 0
    "sol_sym": (1500.0, dict(E1=120e9, E2=8e9, G12=5e9, nu12=0.3, beta=0.01, angles=(0.0, 45.0, 45.0, 0.0))),
    "symm_sol": (1500.0, dict(E1=70e9, G12=5e9, nu12=0.3, beta=0.01, angles=(30.0, -30.0, -30.0, 30.0))),
}


def make_material(name):
    rho, kw = MATERIALS[name]
    atype = "sol" if name == "sol_sym" else name
    return get_material(rho, atype, **kw)


def make_geometry(ny=6, template="sh_i", height=2e-3):
    acc = Accelerometer("AP1030")
    return Geometry(template, acc, GeometryParams(100e-3, 20e-3, height, None, None), ny=ny), acc


def make_problem(material="isotropic", ny=6, **kw):
    from plate_inverse_problem_amd.Problem import Problem
    geom, acc = make_geometry(ny)
    return Problem(geom, make_material(material), acc, **kw)


def oracle_for(p):
    """OracleProblem on the SAME FE data as Problem ``p`` (full reference union pattern)."""
    from oracle.plate_oracle import OracleProblem
    m = p.material
    angles = getattr(m, "angles", None)
    return OracleProblem(p.mat_size, p.rows, p.cols, p.mats, p.vec, np.asarray(p.interp_mat_Lh),
                         np.asarray(p.interp_mat), np.asarray(p.interp_mat_Wx), np.asarray(p.interp_mat_Wy),
                         p.Lh_size, (p.I0, p.I0Corr, p.I2, p.I2Corr), p.accelerometer.height,
                         p.accelerometer.effective_height, p.accelerometer.transverse_sensitivity,
                         m.atype, p.geometry.height, angles)


def report(name, **vals):
    """Measured errors of a GPU test, appended to $PFR_TEST_REPORT (JSON lines) when set."""
    path = os.environ.get("PFR_TEST_REPORT")
    if path:
        import json
        with open(path, "a") as f:
            f.write(json.dumps({"test": name, **{k: [float(x) for x in v] if isinstance(v, (list, tuple)) else float(v)
                                                 for k, v in vals.items()}}) + "\n")
