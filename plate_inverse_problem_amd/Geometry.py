"""Plate geometry and its FE discretisation (``source/jax_plate/Geometry.py``).

The reference copies a FreeFEM ``.edp`` template and regex-substitutes
``Lx, Ly, rAccel, offsetAccelX/Y`` (``Geometry.py:28-238``).  Templates keep the
same names and the same accelerometer placement rules:

* ``'sh_i'``: accelerometer in the corner, centre ``(r, Ly/2 - r)``;
* ``'sh_r'``: custom centre ``(accel_x, Ly/2 - accel_y)``;
* ``'symm'``: centre ``(accel_x, 0)``.

Instead of FreeFEM's mesher the strip is discretised by
``fem.strip_mesh``; ``ny`` (cells across the width) controls the density,
``nx = round(ny * length / width)``.  ``ny = 6`` is the coarse default (about
the reference ``sh_i.edp`` density, 6 boundary segments on the clamped side),
``ny = 12`` gives ~4.6k DOF and ``ny = 25`` ~19.4k DOF.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .Accelerometer import Accelerometer

TEMPLATES = ['sh_r', 'sh_i', 'symm']


@dataclass
class GeometryParams:
    length: float
    width: float
    height: float
    accel_x: float = None
    accel_y: float = None


def dofs_for_density(ny: int, length: float = 100e-3, width: float = 20e-3) -> int:
    """System size ``N = 2 Lh + Mh`` of the strip mesh with ``ny`` cells across."""
    nx = max(1, int(round(ny * length / width)))
    v = (nx + 1) * (ny + 1)
    e = 3 * nx * ny + nx + ny
    return 3 * v + e


class Geometry:
    def __init__(self, edp_or_template: str, accelerometer: Accelerometer = None,
                 params: GeometryParams = None, *, height: float = None,
                 export_vtk: bool = False, ny: int = 6):
        if edp_or_template not in TEMPLATES:
            raise ValueError(f'Could not find template {edp_or_template}. Valid options are: '
                             f'{TEMPLATES}. (FreeFEM .edp scripts are not supported: no FreeFem++ '
                             'binary; the build meshes the strip itself.)')
        if params is None:
            raise ValueError('`params` argument cannot be None when using a template.')
        if accelerometer is None:
            raise ValueError('`accelerometer` argument cannot be None when using a template.')
        params = GeometryParams(**params.__dict__)
        if edp_or_template == 'sh_r':                                        # Geometry.py:89-98
            if None in (params.accel_x, params.accel_y):
                raise ValueError('Both coordinates of accelerometer should be specified for the template sh_r.')
            params.accel_y = params.width / 2 - params.accel_y
        elif edp_or_template == 'sh_i':                                      # :100-108
            if params.accel_y is not None or params.accel_x is not None:
                raise ValueError('Both coordinates of accelerometer should be None for the template sh_i.')
            params.accel_x = accelerometer.radius
            params.accel_y = params.width / 2 - accelerometer.radius
        else:                                                                # :110-119
            if params.accel_y is not None:
                raise ValueError('`y` coordinate of the accelerometer should be None for the template symm.')
            if params.accel_x is None:
                raise ValueError('`x` coordinate of the accelerometer should not be None for the template symm.')
            params.accel_y = 0.0
        if int(ny) < 1:
            raise ValueError('ny must be >= 1')
        self.template = edp_or_template
        self.length = params.length
        self.width = params.width
        self.height = params.height
        self.accel_x = params.accel_x
        self.accel_y = params.accel_y
        self.accel_r = accelerometer.radius
        self.ny = int(ny)
        self.nx = max(1, int(round(self.ny * self.length / self.width)))
        self._ff = None

    @classmethod
    def from_freefem_output(cls, source, height: float, accelerometer: Accelerometer = None) -> "Geometry":
        """A geometry discretised by FreeFem++: ``source`` is the standard output (a path or the text)
        of the reference's matrix-export script -- the geometry's ``.edp`` followed by the varf block
        of ``pyFFInterface.py:175-275`` -- as pyFreeFem reads it (``fem.freefem``).  The 26-matrix
        layout, union pattern and solver then proceed exactly as for a template geometry."""
        from .fem.freefem import load_freefem_output
        ff = load_freefem_output(source)
        g = cls.__new__(cls)
        g.template = 'freefem'
        xy = ff["Th"].vertices
        g.length = float(xy[:, 0].max() - xy[:, 0].min())
        g.width = float(xy[:, 1].max() - xy[:, 1].min())
        g.height = float(height)
        g.accel_x, g.accel_y = float(ff["xtest"]), float(ff["ytest"])
        g.accel_r = accelerometer.radius if accelerometer is not None else None
        g.nx = g.ny = None
        g._ff = ff
        return g

    @property
    def n_dofs(self) -> int:
        if self._ff is not None:
            return 2 * np.asarray(self._ff["vBCLh"]).size + np.asarray(self._ff["vBCMh"]).size
        return dofs_for_density(self.ny, self.length, self.width)

    def build_varfs(self) -> dict:
        """Mesh the strip and assemble every varf of ``pyFFInterface.py:175-275`` (or return the
        FreeFEM-exported ones)."""
        if self._ff is not None:
            return dict(self._ff)
        from .fem import strip_mesh, plate_varfs
        mesh = strip_mesh(self.length, self.width, self.nx, self.ny)
        return plate_varfs(mesh, (self.accel_x, self.accel_y), self.accel_r)

    def __str__(self):
        if self._ff is not None:
            return (f'Geometry from FreeFEM output: {self.length} x {self.width} x {self.height} m, accelerometer '
                    f'at ({self.accel_x}, {self.accel_y}), {self.n_dofs} DOF.')
        return (f'Geometry {self.template}: {self.length} x {self.width} x {self.height} m, '
                f'accelerometer at ({self.accel_x}, {self.accel_y}), mesh {self.nx} x {self.ny} cells.')
