"""Accelerometer parameters (``source/jax_plate/Accelerometer.py:7-115``)."""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, asdict

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))


@dataclass
class AccelerometerParams:
    """mass [kg], radius [m], height [m], effective_height (0..1 along the
    cylinder where the response is measured), transverse_sensitivity (ratio)."""
    mass: float
    radius: float
    height: float
    effective_height: float
    transverse_sensitivity: float


class Accelerometer:
    """Loads ``accelerometers/<name>.json`` or takes an ``AccelerometerParams``."""

    def __init__(self, name_or_params: str | AccelerometerParams):
        if isinstance(name_or_params, str):
            fpath = os.path.join(_PKG_DIR, 'accelerometers', name_or_params + '.json')
            if not os.path.exists(fpath):
                raise ValueError(f'Could not find file {name_or_params}.json in `accelerometers` folder.')
            with open(fpath, 'r') as f:
                params = json.load(f)
        elif isinstance(name_or_params, AccelerometerParams):
            params = asdict(name_or_params)
        else:
            raise TypeError('Argument `name_or_params` should have type `str` or `AccelerometerParams.`')
        self.mass = params['mass']
        self.radius = params['radius']
        self.height = params['height']
        self.effective_height = params['effective_height']
        self.transverse_sensitivity = params['transverse_sensitivity']

    @staticmethod
    def create_accelerometer(params: AccelerometerParams, accelerometer_name: str) -> None:
        folder = os.path.join(_PKG_DIR, 'accelerometers')
        os.makedirs(folder, exist_ok=True)
        with open(os.path.join(folder, accelerometer_name + '.json'), 'w') as f:
            json.dump(asdict(params), f, indent=4)

    def __str__(self):
        return f'Accelerometer with {self.__dict__}.'
