"""Run the REFERENCE's own hot-path code on CPU and record its outputs -> ``reference_run.npz``.

Test data only; run in the build container (``/root/reference`` is not on the GPU box)::

    python tests/golden/make_reference_run.py

JAX is not installed, so the reference modules run under stand-ins that keep their semantics:

* ``jax.numpy`` -> numpy (the closures only use array arithmetic, ``@``, ``mean``, ``abs``,
  ``angle``, ``sqrt``, ``log``, ``einsum``: same float64 / complex128 results); ``jax.jit`` ->
  identity; ``jax.vmap(f, in_axes=(0, None))`` -> a loop over the first argument;
  ``jax.tree_util.Partial`` -> ``functools.partial``;
* the JAX primitive machinery ``Sparse.py`` registers on (``core.Primitive``, ``xla.apply_primitive``,
  ``mlir.register_lowering`` / ``emit_python_callback``) -> a minimal dispatcher, so
  ``spsolve`` -> ``_spsolve_p.bind`` -> the reference's CPU lowering -> its Python callback ->
  ``SolverState.solve`` all run as written;
* the pybind11 ``jax_plate_lib.InnerState`` (UMFPACK; not buildable here: no SuiteSparse) -> the
  oracle's SuperLU factorisation + UMFPACK's default iterative refinement
  (``oracle.plate_oracle.refined_solve``) -- the only non-reference arithmetic in the chain;
* ``jax.value_and_grad`` -> (value, 4th-order central differences of the reference loss)
  for the optimiser runs (JAX's autodiff is not available; the differences are of the reference's
  own loss function), and JAX's immutable arrays are kept immutable (``x -= h * g`` rebinds);
* FreeFem++ -> ``pyFreeFem.edpScript.get_output`` returns this build's varfs on the test mesh
  (as ``make_golden.py`` does); the reference's ``load_matrices_unsymm`` layout, union pattern,
  ``create_symbolic`` / ``find_permutation`` and the unsymmetric ``Problem.__init__`` branch run
  unchanged.

Recorded per material (``ny = 3`` strip, the tests' ``make_problem(material, ny=3)`` mesh):
``Problem.solveForward`` (``Problem.py:611-639`` -> ``getFRFunction`` ``:377-518``), the four
``getLossFunction`` losses (``:933-980``), the central-difference gradient of MSE_LOG_AFC, and
(orthotropic) the trajectories of ``Optimizers.optimize_gd`` / ``optimize_cd``
(``Optimizers.py:231-287``) over 3 steps.  Nothing here unpickles anything; the output is ``np.savez`` arrays.
"""
from __future__ import annotations

import functools
import importlib.util
import os
import sys
import types

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/source"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

FREQS = np.linspace(40.0, 600.0, 24)
LOSSES = ("MSE", "RMSE", "MSE_AFC", "MSE_LOG_AFC")
MATERIALS = ("isotropic", "orthotropic", "orthotropic_d4", "sol")
OPT_MATERIALS = ("orthotropic",)
PERTURB = {"isotropic": [1.05, 0.97, 1.1], "orthotropic": [1.05, 0.97, 1.1, 1.02, 0.95],
           "orthotropic_d4": [1.05, 0.97, 1.1, 1.02, 0.95, 1.04, 1.03, 0.98], "sol": [1.05, 0.97, 1.1, 1.02, 0.95]}


class _JaxArray(np.ndarray):
    """Immutable-update semantics of jax arrays: in-place operators rebind instead of mutating
    (``x -= h * g`` in Optimizers.py must not rewrite the arrays already kept in x_history)."""

    def __isub__(self, o):
        return np.subtract(self, o)

    def __iadd__(self, o):
        return np.add(self, o)


def _fd_grad(f, x, rel=1e-4):
    x = np.asarray(x, dtype=np.float64)
    g = np.zeros_like(x)
    for i in range(x.size):
        h = rel * max(abs(x[i]), 1e-300)
        v = []
        for m in (-2, -1, 1, 2):
            t = np.array(x, dtype=np.float64)
            t[i] += m * h
            v.append(float(f(t.view(_JaxArray))))
        g[i] = (v[0] - 8 * v[1] + 8 * v[2] - v[3]) / (12 * h)
    return g


def _install_standins():
    from oracle.plate_oracle import refined_solve, sparse_lu

    jax = types.ModuleType("jax")
    jax.numpy = np
    jax.Array = np.ndarray
    jax.jit = lambda f, *a, **k: f
    jax.config = types.SimpleNamespace(update=lambda *a, **k: None)

    def vmap(f, in_axes=0):
        def g(xs, *rest):
            return np.array([f(x, *rest) for x in np.asarray(xs)])
        return g
    jax.vmap = vmap

    def value_and_grad(f):
        return lambda x: (float(f(x)), _fd_grad(f, x).view(_JaxArray))
    jax.value_and_grad = value_and_grad
    jax.grad = lambda f: (lambda x: _fd_grad(f, x).view(_JaxArray))
    tu = types.ModuleType("jax.tree_util")
    tu.Partial = functools.partial
    jax.tree_util = tu

    # primitive machinery used by Sparse.py
    core = types.ModuleType("jax.core")

    class Primitive:
        def __init__(self, name):
            self.name = name
            self.impl = None
            self.lowering = None

        def def_impl(self, f):
            self.impl = f

        def def_abstract_eval(self, f):
            self.abstract_eval = f

        def bind(self, *args, **params):
            return self.impl(*args, **params)

    core.Primitive = Primitive
    core.ShapedArray = lambda shape, dtype: (shape, dtype)
    interp = types.ModuleType("jax.interpreters")
    ad = types.ModuleType("jax.interpreters.ad")
    ad.defjvp = lambda *a, **k: None
    ad.primitive_transposes = {}
    ad.is_undefined_primal = lambda x: False
    batching = types.ModuleType("jax.interpreters.batching")
    batching.primitive_batchers = {}
    mlir = types.ModuleType("jax.interpreters.mlir")

    def register_lowering(prim, fn, platform=None):
        prim.lowering = fn

    def emit_python_callback(ctx, callback, token, args, avals_in, avals_out, has_side_effect=False):
        return list(callback(*args)), None, None
    mlir.register_lowering = register_lowering
    mlir.emit_python_callback = emit_python_callback
    xla = types.ModuleType("jax.interpreters.xla")

    def apply_primitive(prim, *args, **params):
        ctx = types.SimpleNamespace(avals_in=None, avals_out=None)
        return prim.lowering(ctx, *args, **params)[0]
    xla.apply_primitive = apply_primitive
    for name, mod in (("ad", ad), ("batching", batching), ("mlir", mlir), ("xla", xla)):
        setattr(interp, name, mod)
        sys.modules["jax.interpreters." + name] = mod
    jax.core = core
    jax.interpreters = interp
    sys.modules.update({"jax": jax, "jax.numpy": np, "jax.tree_util": tu, "jax.core": core,
                        "jax.interpreters": interp})

    # pybind11 InnerState (UMFPACK) -> SuperLU + UMFPACK's default refinement
    lib = types.ModuleType("jax_plate.jax_plate_lib")

    class InnerState:
        def __init__(self):
            self.pat = []

        def add_mat(self, N, indices, indptr, indices_T, indptr_T, perm, data):
            self.pat.append((int(N), np.array(indices), np.array(indptr)))

        def solve(self, data, b, solver_num, transpose, n_cpu, mode):
            if mode != 0:
                raise NotImplementedError("the vmap stand-in only issues unbatched solves")
            N, ind, ptr = self.pat[solver_num]
            A = sp.csc_matrix((np.array(data), ind.copy(), ptr.copy()), shape=(N, N))
            return refined_solve(sparse_lu(A), A, np.asarray(b), trans=bool(transpose))

    lib.InnerState = InnerState
    sys.modules["jax_plate.jax_plate_lib"] = lib
    pkg = types.ModuleType("jax_plate")
    pkg.__path__ = [os.path.join(REF_SRC, "jax_plate")]
    pkg.jax_plate_lib = lib
    sys.modules["jax_plate"] = pkg
    sys.path.insert(0, REF_SRC)           # pyFreeFem


def _load(name):
    path = os.path.join(REF_SRC, "jax_plate", name.split(".")[-1] + ".py")
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def main():
    _install_standins()
    for m in ("Utils", "Accelerometer", "Material", "Geometry", "Input", "pyFFInterface", "Sparse", "Optimizers",
              "Problem"):
        _load("jax_plate." + m)
    import pyFreeFem as pyff
    RP = sys.modules["jax_plate.Problem"]
    RM = sys.modules["jax_plate.Material"]
    RA = sys.modules["jax_plate.Accelerometer"]
    RO = sys.modules["jax_plate.Optimizers"]
    from helpers import MATERIALS as MATS, make_geometry

    geom, _ = make_geometry(ny=3)
    ff = geom.build_varfs()
    edp = os.path.join(REF_SRC, "jax_plate", "geometry", "sh_i.edp")
    out = {"freqs": FREQS}
    orig = pyff.edpScript.get_output
    pyff.edpScript.get_output = lambda self, *a, **k: dict(ff)
    try:
        for name in MATERIALS:
            rho, kw = MATS[name]
            mat = RM.get_material(rho, "sol" if name == "sol_sym" else name, **kw)
            acc = RA.Accelerometer("AP1030")
            g = types.SimpleNamespace(current_file=edp, height=geom.height)
            prob = RP.Problem(g, mat, acc)
            theta0 = np.asarray(prob.parameters, dtype=np.float64)
            fr = np.asarray(prob.solveForward(FREQS), dtype=np.float64)
            ref = fr * np.exp(0.1j) * 1.02
            theta = theta0 * np.array(PERTURB[name])
            out[f"{name}_theta0"] = theta0
            out[f"{name}_theta"] = theta
            out[f"{name}_fr"] = fr
            out[f"{name}_ref"] = ref
            for lt in LOSSES:
                f = prob.getLossFunction(FREQS, ref, lt)
                out[f"{name}_{lt}_loss"] = np.float64(f(theta.view(_JaxArray)))
            # central differences of the reference loss in scaled parameters (x = theta / theta0)
            fs = prob.getLossFunction(FREQS, ref, "MSE_LOG_AFC", theta0)
            out[f"{name}_MSE_LOG_AFC_grad_scaled"] = _fd_grad(fs, (theta / theta0).view(_JaxArray), rel=1e-4)
            if name in OPT_MATERIALS:
                # optimiser trajectories on the scaled MSE_LOG_AFC loss (solveInverse use_scaling form)
                x0 = (theta / theta0).view(_JaxArray)
                for opt, fn, kw_ in (("gd", RO.optimize_gd, dict(N_steps=3, h=0.05)),
                                     ("cd", RO.optimize_cd, dict(N_steps=3, h=0.05))):
                    res = fn(fs, x0.copy().view(_JaxArray), **kw_)
                    out[f"{name}_{opt}_x"] = np.array([np.asarray(v, dtype=np.float64) for v in res.x_history + [res.x]])
                    out[f"{name}_{opt}_f"] = np.array([float(v) for v in res.f_history + [res.f]])
            print(name, "fr[0..3]", fr[:3], "MSE_LOG_AFC", out[f"{name}_MSE_LOG_AFC_loss"], flush=True)
    finally:
        pyff.edpScript.get_output = orig
    np.savez_compressed(os.path.join(HERE, "reference_run.npz"), **out)
    print("reference_run.npz")


if __name__ == "__main__":
    main()
