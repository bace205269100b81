"""plate_inverse_problem_amd -- MI355X-native differentiable plate frequency-response solver.

Keeps the reference ``jax_plate`` API (``Problem``, ``getFRFunction`` /
``getAFCFunction``, ``solveForward`` / ``solve_forward``, ``getLossFunction``,
``solveInverse``) on top of hand-written HIP kernels (``csrc/``, C ABI in
``include/pfr.h``) driven from PyTorch-ROCm.
"""
from . import Accelerometer, Geometry, Material  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # heavy modules (torch autograd functions, FE assembly) load on first use
    import importlib
    if name in ("Problem", "Sparse", "Optimizers", "Input", "distributed", "fem", "inverse"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
