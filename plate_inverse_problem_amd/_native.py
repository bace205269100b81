"""ctypes binding of ``libpfr.so`` (C ABI declared in ``include/pfr.h``).

This is the reference-side binding a maintainer would add in place of the
pybind11 module ``jax_plate_lib`` (``source/jax_plate_lib/src/main.cpp:4-20``,
used by ``SolverState`` at ``source/jax_plate/Sparse.py:19-44``).

The library is built in-tree (``plate_inverse_problem_amd/_lib/libpfr.so``) by
``__graft_entry__.build()``; there is no CPU fallback: every compute entry
point raises if the library is missing or a call fails.
"""
from __future__ import annotations

import ctypes as C
import os
import re

import numpy as np

LIB_PATH = os.environ.get("PFR_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libpfr.so")
HEADER_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "pfr.h")

PFR_OK = 0
PFR_FLAG_BAD_PIVOT = 1
PFR_FLAG_BACKWARD_ERROR = 2
PFR_FLAG_BACKWARD_ERROR_ADJ = 4
PFR_CHECK_FORWARD, PFR_CHECK_ADJOINT, PFR_CHECK_REFINE, PFR_CHECK_CORRECT = 1, 2, 4, 8
PFR_CHECK_REFINE_ADJ = 16
LOSS_NONE, LOSS_MSE, LOSS_RMSE, LOSS_MSE_AFC, LOSS_MSE_LOG_AFC, LOSS_COTANGENT = -1, 0, 1, 2, 3, 4
LOSS_IDS = {"MSE": LOSS_MSE, "RMSE": LOSS_RMSE, "MSE_AFC": LOSS_MSE_AFC, "MSE_LOG_AFC": LOSS_MSE_LOG_AFC}

EXPORT = dict(PERM=0, IPERM=1, FRONTS=2, IDX=3, RELPOS=4, ASM_PTR=5, ASM_COL=6, ASM_NZ=7, EA_PTR=8,
              EA_SRC=9, LEVEL_PTR=10, LEVEL_FRONTS=11, DIRICHLET=12, COUPLING=13)


class NativeError(RuntimeError):
    pass


class SymbolicOptions(C.Structure):
    _fields_ = [("leaf_size", C.c_int32), ("ordering", C.c_int32), ("relax_small", C.c_int32),
                ("relax_mid", C.c_int32), ("relax_big", C.c_int32), ("zrelax_mid", C.c_double),
                ("zrelax_big", C.c_double), ("symmetric", C.c_int32), ("n_last", C.c_int32),
                ("last", C.POINTER(C.c_int32)), ("max_ns", C.c_int32), ("md_delta", C.c_int32)]


class SymbolicStats(C.Structure):
    _fields_ = [("n", C.c_int32), ("nnz", C.c_int64), ("n_fronts", C.c_int32), ("n_levels", C.c_int32),
                ("max_front", C.c_int32), ("total_rows", C.c_int64), ("factor_entries", C.c_int64),
                ("nnz_lu", C.c_int64), ("factor_flops", C.c_double), ("symmetric", C.c_int32),
                ("n_dirichlet", C.c_int32), ("n_coupling", C.c_int64)]


_P = C.c_void_p
_I32P = C.POINTER(C.c_int32)
_DP = C.POINTER(C.c_double)

_PROTOS = {
    "pfr_version": (C.c_char_p, []),
    "pfr_last_error": (C.c_char_p, []),
    "pfr_symbolic_options_default": (None, [C.POINTER(SymbolicOptions)]),
    "pfr_symbolic_create": (C.c_int, [C.c_int32, C.c_int64, _I32P, _I32P, C.POINTER(SymbolicOptions), C.POINTER(_P)]),
    "pfr_symbolic_stats_get": (C.c_int, [_P, C.POINTER(SymbolicStats)]),
    "pfr_symbolic_export": (C.c_int, [_P, C.c_int32, _P, C.c_int64]),
    "pfr_symbolic_destroy": (None, [_P]),
    "pfr_solver_create": (C.c_int, [_P, _I32P, _I32P, C.c_int32, C.c_int32, C.POINTER(_P)]),
    "pfr_solver_destroy": (None, [_P]),
    "pfr_solver_workspace_bytes": (C.c_int64, [_P, C.c_int32]),
    "pfr_solver_max_batch": (C.c_int32, [_P]),
    "pfr_solve": (C.c_int, [_P, C.c_int32, _P, C.c_int64, _P, C.c_int64, _P, C.c_int32, _P, _P]),
    "pfr_matvec": (C.c_int, [_P, C.c_int32, _P, C.c_int64, _P, C.c_int64, _P, C.c_int32, _P]),
    "pfr_set_stiffness": (C.c_int, [_P, C.c_int32, _P, _DP]),
    "pfr_combine": (C.c_int, [_P, _DP, _P, _P]),
    "pfr_set_operator": (C.c_int, [_P, _P, _P]),
    "pfr_set_rhs": (C.c_int, [_P, _DP, C.c_double, C.c_double, C.c_double]),
    "pfr_set_functional": (C.c_int, [_P, C.c_int32, _I32P, _DP, C.c_double]),
    "pfr_sweep": (C.c_int, [_P, C.c_int32, _P, C.c_int32, _P, C.c_double, _P, _P, _P, _P, _P]),
    "pfr_sweep_graph_launches": (C.c_int64, [_P]),
    "pfr_stream_order": (C.c_int, [_P, _P]),
    "pfr_sweep_fresh": (C.c_int, [_P, C.c_int32, _P, C.c_int32, _P, C.c_double, _P, _P, _P, _P, _P]),
    "pfr_solve_multi": (C.c_int, [_P, C.c_int32, C.c_int32, _P, C.c_int64, _P, C.c_int64, C.c_int64, _P, C.c_int64,
                                  C.c_int32, _P, _P]),
    "pfr_hessian_sweep": (C.c_int, [_P, C.c_int32, _P, C.c_int32, _P, C.c_double, C.c_int32, _P, _P, _P, _P, _P,
                                    _P]),
    "pfr_set_check": (C.c_int, [_P, C.c_int32, C.c_double, _P]),
    "pfr_set_refine_tol": (C.c_int, [_P, C.c_double]),
    "pfr_debug_solution": (C.c_int, [_P, C.c_int32, C.c_int32, _DP]),
    "pfr_set_timing": (C.c_int, [_P, C.c_int32]),
    "pfr_last_timings": (C.c_int, [_P, _DP]),
    "pfr_last_kernel_timings": (C.c_int, [_P, _DP, _P]),
    "pfr_solver_alg_bytes": (C.c_int, [_P, _P]),
    "pfr_solver_solve_bytes": (C.c_int, [_P, _P]),
}

_lib = None


def header_symbols() -> list[str]:
    """Function names declared ``PFR_API`` in include/pfr.h."""
    with open(HEADER_PATH) as f:
        txt = f.read()
    return re.findall(r"PFR_API\s+[\w\s\*]+?\b(pfr_\w+)\s*\(", txt)


def lib():
    """Load libpfr.so (once).  Raises NativeError if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                          " (no CPU fallback exists for the solver path)")
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != PFR_OK:
        msg = lib().pfr_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (status {rc}): {msg}")


def _i32(a):
    a = np.ascontiguousarray(a, dtype=np.int32)
    return a, a.ctypes.data_as(_I32P)


def _f64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_DP)


def _ptr(t) -> int:
    """Device pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return None
    if not t.is_contiguous():
        raise ValueError("device tensors passed to libpfr must be contiguous")
    return t.data_ptr()


def stream_order(waiter: int, signaller: int):
    """pfr_stream_order: work enqueued on HIP stream ``waiter`` from now on runs after the work enqueued on
    ``signaller`` so far (stream handles, e.g. torch.cuda.Stream.cuda_stream)."""
    check(lib().pfr_stream_order(waiter, signaller), "pfr_stream_order")


class Symbolic:
    """Host-only symbolic analysis (nested dissection + supernodal maps)."""

    def __init__(self, n: int, colptr, rowind, *, leaf_size=None, ordering=0, relax=None, symmetric=False,
                 last=None, max_ns=None, md_delta=None):
        L = lib()
        opt = SymbolicOptions()
        L.pfr_symbolic_options_default(C.byref(opt))
        if leaf_size is not None:
            opt.leaf_size = int(leaf_size)
        opt.ordering = int(ordering)
        opt.symmetric = int(bool(symmetric))
        if max_ns is not None:
            opt.max_ns = int(max_ns)
        if md_delta is not None:
            opt.md_delta = int(md_delta)
        if last is not None and len(last):
            self.last, lp = _i32(last)
            opt.n_last = int(self.last.size)
            opt.last = lp
        if relax is not None:
            opt.relax_small, opt.relax_mid, opt.relax_big = (int(v) for v in relax[:3])
            if len(relax) > 3:
                opt.zrelax_mid, opt.zrelax_big = (float(v) for v in relax[3:5])
        self.colptr, cp = _i32(colptr)
        self.rowind, ri = _i32(rowind)
        self.n = int(n)
        h = _P()
        check(L.pfr_symbolic_create(self.n, int(self.rowind.size), cp, ri, C.byref(opt), C.byref(h)),
              "pfr_symbolic_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def stats(self) -> dict:
        st = SymbolicStats()
        check(lib().pfr_symbolic_stats_get(self._h, C.byref(st)), "pfr_symbolic_stats_get")
        return {k: getattr(st, k) for k, _ in SymbolicStats._fields_}

    def export(self, what: str) -> np.ndarray:
        st = self.stats()
        sizes = {"PERM": st["n"], "IPERM": st["n"], "FRONTS": 8 * st["n_fronts"], "IDX": st["total_rows"],
                 "RELPOS": st["total_rows"], "ASM_PTR": st["total_rows"] + 1, "ASM_COL": st["nnz"],
                 "ASM_NZ": st["nnz"], "EA_PTR": st["total_rows"] + 1, "LEVEL_PTR": st["n_levels"] + 1,
                 "LEVEL_FRONTS": st["n_fronts"]}
        if what == "EA_SRC":
            size = int(self.export("EA_PTR")[-1])
        elif what == "DIRICHLET":
            size = 2 * st["n_dirichlet"]
        elif what == "COUPLING":
            size = 3 * st["n_coupling"]
        elif what in ("ASM_COL", "ASM_NZ"):
            size = int(self.export("ASM_PTR")[-1])
        else:
            size = sizes[what]
        dtype = np.int64 if what == "FRONTS" else np.int32
        out = np.zeros(size, dtype=dtype)
        check(lib().pfr_symbolic_export(self._h, EXPORT[what], out.ctypes.data_as(_P), out.nbytes),
              "pfr_symbolic_export")
        if what == "FRONTS":
            return out.reshape(-1, 8)
        if what == "DIRICHLET":
            return out.reshape(-1, 2)
        if what == "COUPLING":
            return out.reshape(-1, 3)
        return out

    def workspace_bytes(self, max_batch: int) -> int:
        return int(lib().pfr_solver_workspace_bytes(self._h, int(max_batch)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.pfr_symbolic_destroy(h)
            self._h = None


class Solver:
    """Device-resident batched solver for one pattern (one per device)."""

    def __init__(self, sym: Symbolic, device_index: int, max_batch: int):
        L = lib()
        self.sym = sym
        self.device_index = int(device_index)
        h = _P()
        _, cp = _i32(sym.colptr)
        _, ri = _i32(sym.rowind)
        check(L.pfr_solver_create(sym.handle, cp, ri, self.device_index, int(max_batch), C.byref(h)),
              "pfr_solver_create")
        self._h = h
        self.max_batch = int(L.pfr_solver_max_batch(h))
        self._keep = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and _lib is not None:
            _lib.pfr_solver_destroy(h)
            self._h = None

    @staticmethod
    def _stream(t):
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream

    # ---- operator-form state
    def set_stiffness(self, stiff_nz_k, rhs_weights):
        self._keep["stiff"] = stiff_nz_k
        w, wp = _f64(rhs_weights)
        check(lib().pfr_set_stiffness(self._h, int(stiff_nz_k.shape[1]), _ptr(stiff_nz_k), wp), "pfr_set_stiffness")

    def combine(self, coef: np.ndarray, out):
        c = np.ascontiguousarray(np.asarray(coef, dtype=np.complex128))
        check(lib().pfr_combine(self._h, c.view(np.float64).ctypes.data_as(_DP), _ptr(out), self._stream(out)),
              "pfr_combine")
        return out

    def set_operator(self, K, M):
        self._keep["K"], self._keep["M"] = K, M
        check(lib().pfr_set_operator(self._h, _ptr(K), _ptr(M)), "pfr_set_operator")

    def set_rhs(self, rhs, beta: complex, mass_sum: float):
        r, rp = _f64(rhs)
        check(lib().pfr_set_rhs(self._h, rp, float(np.real(beta)), float(np.imag(beta)), float(mass_sum)),
              "pfr_set_rhs")

    def set_functional(self, index, a3, ts: float):
        i, ip = _i32(index)
        a, ap = _f64(np.asarray(a3).reshape(-1))
        check(lib().pfr_set_functional(self._h, int(i.size), ip, ap, float(ts)), "pfr_set_functional")

    def sweep(self, freqs, loss_type=LOSS_NONE, ref=None, scale=1.0, fr=None, loss=None, w=None, flags=None,
              fresh=False, stream=None):
        """pfr_sweep (loss / w / flags accumulated into), or with ``fresh`` pfr_sweep_fresh (they and the
        pfr_set_check backward errors initialised by the sweep's first kernel); on ``stream`` (a HIP stream
        handle) or the current torch stream."""
        fn = lib().pfr_sweep_fresh if fresh else lib().pfr_sweep
        check(fn(self._h, int(freqs.numel()), _ptr(freqs), int(loss_type), _ptr(ref), float(scale),
                 _ptr(fr), _ptr(loss), _ptr(w), _ptr(flags), self._stream(freqs) if stream is None else stream),
              "pfr_sweep")

    def hessian_sweep(self, freqs, loss_type, ref, scale, dcoef, loss=None, w=None, h=None, flags=None):
        """Loss, gradient partials w (18 complex) and second-order partials h (n_dir x 18 complex) with the
        factors reused for the tangent and second-order adjoint solves; ``dcoef`` (n_dir, n_stiff) complex
        host array of coefficient directions d c / d theta_i."""
        d = np.ascontiguousarray(np.asarray(dcoef, dtype=np.complex128))
        check(lib().pfr_hessian_sweep(self._h, int(freqs.numel()), _ptr(freqs), int(loss_type), _ptr(ref),
                                      float(scale), int(d.shape[0]), d.ctypes.data_as(_P), _ptr(loss), _ptr(w),
                                      _ptr(h), _ptr(flags), self._stream(freqs)), "pfr_hessian_sweep")

    # ---- InnerState-compatible
    def solve(self, data, data_stride, b, b_stride, x, transpose, batch, flags=None):
        check(lib().pfr_solve(self._h, int(batch), _ptr(data), int(data_stride), _ptr(b), int(b_stride), _ptr(x),
                              int(bool(transpose)), _ptr(flags), self._stream(x)), "pfr_solve")

    def solve_multi(self, data, data_stride, b, b_stride, b_rhs_stride, x, x_rhs_stride, transpose, batch, nrhs,
                    flags=None):
        check(lib().pfr_solve_multi(self._h, int(batch), int(nrhs), _ptr(data), int(data_stride), _ptr(b),
                                    int(b_stride), int(b_rhs_stride), _ptr(x), int(x_rhs_stride),
                                    int(bool(transpose)), _ptr(flags), self._stream(x)), "pfr_solve_multi")

    def matvec(self, data, data_stride, x, x_stride, y, transpose, batch):
        check(lib().pfr_matvec(self._h, int(batch), _ptr(data), int(data_stride), _ptr(x), int(x_stride), _ptr(y),
                               int(bool(transpose)), self._stream(y)), "pfr_matvec")

    # ---- backward-error checks
    def debug_solution(self, which: int, q: int) -> np.ndarray:
        """The last chunk's forward solution (0) or adjoint (1) of chunk lane q, caller numbering (diagnostic)."""
        out = np.zeros(2 * self.sym.stats()["n"], dtype=np.float64)
        check(lib().pfr_debug_solution(self._h, int(which), int(q), out.ctypes.data_as(_DP)), "pfr_debug_solution")
        return out[0::2] + 1j * out[1::2]

    def set_refine_tol(self, tol: float):
        """Threshold of the selective adjoint refinement (PFR_CHECK_REFINE_ADJ): groups where the functional
        correction exceeds tol |fr| get one refinement step of the fr adjoint."""
        check(lib().pfr_set_refine_tol(self._h, float(tol)), "pfr_set_refine_tol")

    def set_check(self, mode: int, tol: float, berr=None):
        """PFR_CHECK_* bits, flag tolerance; ``berr`` (device float64, 2 per frequency of each later
        call, or None) receives the componentwise backward errors (forward, adjoint)."""
        check(lib().pfr_set_check(self._h, int(mode), float(tol), _ptr(berr)), "pfr_set_check")

    def graph_launches(self) -> int:
        """Sweeps of this solver replayed from its captured hipGraph (pfr_sweep_graph_launches)."""
        return int(lib().pfr_sweep_graph_launches(self._h))

    # ---- timing
    def set_timing(self, on, kernels: bool = False):
        """Per-phase HIP-event timing; ``kernels`` also brackets every factorisation launch."""
        check(lib().pfr_set_timing(self._h, (3 if kernels else 1) if on else 0), "pfr_set_timing")

    def last_timings(self) -> np.ndarray:
        out = np.zeros(5)
        check(lib().pfr_last_timings(self._h, out.ctypes.data_as(_DP)), "pfr_last_timings")
        return out

    KERNEL_CLASSES = ("k_assemble_level", "k_factor_level", "k_offdiag_level", "k_schur_sym_blk", "k_schur_level")

    def last_kernel_timings(self):
        """(ms, launches) per factorisation kernel class of the last call (needs kernels=True)."""
        ms = np.zeros(5)
        n = np.zeros(5, np.int64)
        check(lib().pfr_last_kernel_timings(self._h, ms.ctypes.data_as(_DP), n.ctypes.data_as(_P)),
              "pfr_last_kernel_timings")
        return ms, n

    def alg_bytes(self) -> np.ndarray:
        """Algorithmic HBM bytes per frequency of one factorisation, per kernel class."""
        out = np.zeros(5, np.int64)
        check(lib().pfr_solver_alg_bytes(self._h, out.ctypes.data_as(_P)), "pfr_solver_alg_bytes")
        return out

    def solve_bytes(self) -> np.ndarray:
        """Algorithmic HBM bytes per frequency of the forward and the adjoint solve pair of a sweep."""
        out = np.zeros(2, np.int64)
        check(lib().pfr_solver_solve_bytes(self._h, out.ctypes.data_as(_P)), "pfr_solver_solve_bytes")
        return out
