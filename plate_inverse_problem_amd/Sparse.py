"""Batched sparse solve / matvec primitives with autograd (``source/jax_plate/Sparse.py``).

The reference registers JAX primitives ``cpu_spsolve`` / ``custom_matvec``
whose CPU lowering calls the pybind11 ``InnerState`` (UMFPACK, OpenMP over the
batch).  Here the same entry points are torch autograd functions over the C ABI
(``pfr_solve`` / ``pfr_matvec``, HIP, frequency-minor batched multifrontal LU):

* ``create_symbolic(N, indices, dtype)`` -> ``((rows, cols), solver_num)``
  (``Sparse.py:92-116``): symbolic analysis once per pattern; the returned
  coordinates are the CSC order ``data`` must follow;
* ``spsolve(data, b, solver_num=, transpose=)`` (``Sparse.py:231-236``): batching
  by shape like the reference's modes (``Sparse.py:238-277``): data ``(nnz,)`` or
  ``(B, nnz)``, b ``(N,)``, ``(B, N)`` or ``(J, B, N)`` (mode 4);
  ``transpose=True`` solves with the NON-conjugate transpose (``UMFPACK_Aat``);
* ``matvec(data, vec, solver_num=, transpose=)`` (``Sparse.py:144-183``).

Gradients follow torch's conjugate-Wirtinger convention (``torch.linalg.solve``):
``gb = A^{-H} gx``, ``gA[k] = -gb[row_k] conj(x[col_k])``.
"""
from __future__ import annotations

import warnings
from multiprocessing import cpu_count

import numpy as np
import torch

from . import _native


class SolverState:
    """Registry of symbolic analyses (``Sparse.py:19-44``); one device solver each."""

    def __init__(self):
        self.patterns = []
        self.permutations = []
        self._entries = []

    @property
    def state_size(self) -> int:
        return len(self.patterns)

    def add_mat(self, N: int, rows: np.ndarray, cols: np.ndarray, device=None, max_batch=None) -> int:
        order = np.lexsort((rows, cols))                 # CSC: by column, then row
        r, c = rows[order].astype(np.int32), cols[order].astype(np.int32)
        colptr = np.zeros(N + 1, dtype=np.int64)
        np.add.at(colptr, c.astype(np.int64) + 1, 1)
        colptr = np.cumsum(colptr).astype(np.int32)
        sym = _native.Symbolic(N, colptr, r)
        self.patterns.append(np.stack([r, c], axis=1))
        self.permutations.append(order)
        self._entries.append(dict(sym=sym, N=N, nnz=r.size, device=device, max_batch=max_batch, solver=None,
                                  rows=torch.as_tensor(r.astype(np.int64)), cols=torch.as_tensor(c.astype(np.int64))))
        return self.state_size - 1

    def solver(self, num: int, device: torch.device, batch: int) -> _native.Solver:
        e = self._entries[num]
        if e["solver"] is None:
            mb = e["max_batch"] or max(64, min(1024, (batch + 63) // 64 * 64))
            e["solver"] = _native.Solver(e["sym"], device.index, mb)
            # UMFPACK's default solve (the reference passes a NULL Control) refines up to 2 steps; the
            # static pivot order here gets one refinement step and a backward-error check of every solve
            e["solver"].set_check(CHECK_MODE, CHECK_TOL)
        return e["solver"]

    def entry(self, num: int) -> dict:
        return self._entries[num]


_SOLVER_STATE = SolverState()
CHECK_MODE = _native.PFR_CHECK_FORWARD | _native.PFR_CHECK_ADJOINT | _native.PFR_CHECK_REFINE
CHECK_TOL = 1e-10


def _flags(flags):
    """Bad static pivot -> error (UMFPACK reports a singular matrix as an error status,
    umfpack_interface.h:10-18); backward error above the tolerance after refinement -> warning."""
    f = flags.cpu().numpy()
    if (f & _native.PFR_FLAG_BAD_PIVOT).any():
        raise _native.NativeError("zero/non-finite static pivot in spsolve (matrix singular in the fixed order)")
    bad = int(np.count_nonzero(f & (_native.PFR_FLAG_BACKWARD_ERROR | _native.PFR_FLAG_BACKWARD_ERROR_ADJ)))
    if bad:
        warnings.warn(f"spsolve: {bad} of {f.size} solves keep a componentwise backward error above {CHECK_TOL:g} "
                      "after refinement (static pivot order unstable for these matrices)", RuntimeWarning)


def create_symbolic(N: int, indices: np.ndarray, mat_dtype=np.complex128, *, device=None, max_batch=None):
    """Symbolic analysis of an ``N x N`` pattern given as ``(nnz, 2)`` (row, col) pairs."""
    indices = np.asarray(indices)
    if indices.ndim != 2 or indices.shape[1] != 2:
        raise TypeError("indices must have shape (nnz, 2)")
    if np.dtype(mat_dtype) not in (np.dtype(np.float64), np.dtype(np.complex128)):
        raise TypeError(f"Invalid dtype {mat_dtype}: expected float64 or complex128")
    num = _SOLVER_STATE.add_mat(int(N), indices[:, 0], indices[:, 1], device, max_batch)
    patt = _SOLVER_STATE.patterns[num]
    return (patt[:, 0], patt[:, 1]), num


def _check(data, b, solver_num, n_cpu, _mode):
    if not isinstance(solver_num, int):
        raise TypeError(f"invalid type of `solver_num` argument, expected `int`, got {type(solver_num)}")
    if n_cpu is not None and (not isinstance(n_cpu, int) or n_cpu < 0):
        raise ValueError("n_cpu argument should be a non-negative int")
    if data.dtype != b.dtype:
        raise ValueError(f"data types do not match: {data.dtype=} {b.dtype=}")
    if data.device.type != "cuda":
        raise _native.NativeError("spsolve/matvec run on the ROCm device only (no CPU fallback)")


def _as_c(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.complex128).contiguous()


def _raw_solve(num, data, b, transpose):
    """data (nnz,) or (B, nnz); b (B, N) complex; returns (B, N)."""
    data, b = data.resolve_conj().contiguous(), b.resolve_conj().contiguous()
    e = _SOLVER_STATE.entry(num)
    B = b.shape[0]
    s = _SOLVER_STATE.solver(num, b.device, B)
    ds = 0 if data.dim() == 1 else e["nnz"]
    x = torch.empty_like(b)
    flags = torch.zeros(B, dtype=torch.int32, device=b.device)
    s.solve(torch.view_as_real(data), ds, torch.view_as_real(b), e["N"], torch.view_as_real(x), transpose, B, flags)
    _flags(flags)
    return x


def _raw_solve_multi(num, data, b, transpose):
    """data (nnz,) or (B, nnz); b (J, B, N) complex; every right-hand side on the same factors."""
    data, b = data.resolve_conj().contiguous(), b.resolve_conj().contiguous()
    e = _SOLVER_STATE.entry(num)
    J, B = b.shape[0], b.shape[1]
    s = _SOLVER_STATE.solver(num, b.device, B)
    ds = 0 if data.dim() == 1 else e["nnz"]
    x = torch.empty_like(b)
    flags = torch.zeros(B, dtype=torch.int32, device=b.device)
    s.solve_multi(torch.view_as_real(data), ds, torch.view_as_real(b), e["N"], B * e["N"], torch.view_as_real(x),
                  B * e["N"], transpose, B, J, flags)
    _flags(flags)
    return x


def _raw_matvec(num, data, v, transpose):
    data, v = data.resolve_conj().contiguous(), v.resolve_conj().contiguous()
    e = _SOLVER_STATE.entry(num)
    B = v.shape[0]
    s = _SOLVER_STATE.solver(num, v.device, B)
    ds = 0 if data.dim() == 1 else e["nnz"]
    y = torch.empty_like(v)
    s.matvec(torch.view_as_real(data), ds, torch.view_as_real(v), e["N"], torch.view_as_real(y), transpose, B)
    return y


class _Solve(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, b, num, transpose):
        x = _raw_solve(num, data, b, transpose)
        ctx.save_for_backward(data, x)
        ctx.num, ctx.transpose = num, transpose
        return x

    @staticmethod
    def backward(ctx, gx):
        data, x = ctx.saved_tensors
        e = _SOLVER_STATE.entry(ctx.num)
        gb = torch.conj(_raw_solve(ctx.num, data, torch.conj(gx).contiguous(), not ctx.transpose))
        rows, cols = e["rows"].to(x.device), e["cols"].to(x.device)
        if ctx.transpose:
            rows, cols = cols, rows
        gA = -(gb[:, rows] * torch.conj(x[:, cols]))
        if data.dim() == 1:
            gA = gA.sum(0)
        return gA, gb, None, None


class _SolveMulti(torch.autograd.Function):
    """Mode 4: b (J, B, N), data (B, nnz) or (nnz,); one factorisation per matrix."""

    @staticmethod
    def forward(ctx, data, b, num, transpose):
        x = _raw_solve_multi(num, data, b, transpose)
        ctx.save_for_backward(data, x)
        ctx.num, ctx.transpose = num, transpose
        return x

    @staticmethod
    def backward(ctx, gx):
        data, x = ctx.saved_tensors
        e = _SOLVER_STATE.entry(ctx.num)
        gb = torch.conj(_raw_solve_multi(ctx.num, data, torch.conj(gx).contiguous(), not ctx.transpose))
        rows, cols = e["rows"].to(x.device), e["cols"].to(x.device)
        if ctx.transpose:
            rows, cols = cols, rows
        gA = -(gb[:, :, rows] * torch.conj(x[:, :, cols])).sum(0)
        if data.dim() == 1:
            gA = gA.sum(0)
        return gA, gb, None, None


class _Matvec(torch.autograd.Function):
    @staticmethod
    def forward(ctx, data, v, num, transpose):
        y = _raw_matvec(num, data, v, transpose)
        ctx.save_for_backward(data, v)
        ctx.num, ctx.transpose = num, transpose
        return y

    @staticmethod
    def backward(ctx, gy):
        data, v = ctx.saved_tensors
        e = _SOLVER_STATE.entry(ctx.num)
        gv = torch.conj(_raw_matvec(ctx.num, data, torch.conj(gy).contiguous(), not ctx.transpose))
        rows, cols = e["rows"].to(v.device), e["cols"].to(v.device)
        if ctx.transpose:
            rows, cols = cols, rows
        gA = gy[:, rows] * torch.conj(v[:, cols])
        if data.dim() == 1:
            gA = gA.sum(0)
        return gA, gv, None, None


def _batched(fn, data, b, solver_num, transpose):
    real = not torch.is_complex(b)
    d, v = _as_c(data), _as_c(b)
    if v.dim() == 1:                                     # modes 0 / 1
        if d.dim() == 2:
            out = fn(d, v.unsqueeze(0).expand(d.shape[0], -1).contiguous(), solver_num, transpose)
        else:
            out = fn(d, v.unsqueeze(0), solver_num, transpose)[0]
    elif v.dim() == 2:                                   # modes 2 / 3
        out = fn(d, v, solver_num, transpose)
    elif v.dim() == 3:                                   # mode 4: b (J, B, N), data (B, nnz)
        if fn is _Solve.apply:                           # all J right-hand sides on the same factors
            out = _SolveMulti.apply(d, v.contiguous(), solver_num, transpose)
        else:
            out = torch.stack([fn(d, v[j], solver_num, transpose) for j in range(v.shape[0])])
    else:
        raise NotImplementedError(f"Batching of spsolve with arguments shapes: {data.shape=}, {b.shape=}")
    return out.real if real else out


def spsolve(data, b, *, solver_num: int, transpose: bool = False, n_cpu=None, _mode=None):
    """A sparse direct solve on the device (``Sparse.py:231``); ``n_cpu`` is accepted
    for signature compatibility (0 -> cpu_count(), as the reference) and ignored."""
    if n_cpu == 0:
        n_cpu = cpu_count()
    _check(data, b, solver_num, n_cpu, _mode)
    return _batched(_Solve.apply, data, b, solver_num, bool(transpose))


def matvec(mat, vec, *, solver_num: int, transpose: bool = False, n_cpu=None, _mode=None):
    """Batched CSC matrix-vector product (``Sparse.py:144``)."""
    if n_cpu == 0:
        n_cpu = cpu_count()
    _check(mat, vec, solver_num, n_cpu, _mode)
    return _batched(_Matvec.apply, mat, vec, solver_num, bool(transpose))
