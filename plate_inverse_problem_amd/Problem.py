"""``Problem``: differentiable plate frequency response on MI355X.

Mirrors ``source/jax_plate/Problem.py`` (constructor semantics, ``getFRFunction``,
``solveForward``, ``getLossFunction``, ``solveInverse``) -- the unsymmetric
(accelerometer) branch, which is the reference's only live branch (SURVEY.md
§2).  The reference's JAX ``jit(vmap(_solve))`` + UMFPACK-callback hot path is
replaced by one fused HIP sweep per frequency chunk (``_native.Solver.sweep``):

    assemble K(theta) - omega^2 M -> static-pivot multifrontal LU -> L/U solves
    -> FR functional [-> loss cotangent -> U^T/L^T adjoint solves ->
    stiffness contraction]

Autodiff: the sweep is a ``torch.autograd.Function`` of the 18 complex laminate
coefficients ``c = (A, B, D)``; torch autograd carries the gradient through the
material transform to ``theta``.  Gradients are exact adjoints (no finite
differences), with the reference's non-conjugate transpose (``Sparse.py:211-219``).
"""
from __future__ import annotations

import json
import os
import warnings
import weakref
from typing import Callable

import numpy as np
import scipy.sparse as sp
import torch

from . import _native
from ._abd_jet import coeffs18 as _jet_coeffs18, _cached_abd
from .Accelerometer import Accelerometer, AccelerometerParams
from .Geometry import Geometry, GeometryParams
from .Material import Material, get_material
from .fem.layout import load_matrices_unsymm, union_pattern

RHS_WEIGHTS_D = np.array([1.0, 2.0, 4.0, 1.0, 4.0, 4.0])   # Problem.py:447-448
KB_SLICE = slice(6, 12)                                     # the 6 coupling (B) matrices
_PKG_DIR = os.path.dirname(os.path.abspath(__file__))


def _default_device():
    if not torch.cuda.is_available():
        raise _native.NativeError("the plate solver runs on a ROCm GPU; torch.cuda.is_available() is False "
                                  "(there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def decoupled_symmetric(rows, cols, vals, n, rtol=1e-10) -> bool:
    """True when every matrix ``vals[k]`` on the (rows, cols) pattern is complex symmetric
    once the Dirichlet rows -- rows holding only their diagonal entry, the ``tgv = -1`` rows
    of pyFFInterface.py:176 -- and their columns are taken out (the condition of the
    symmetric analysis, include/pfr.h ``pfr_symbolic_options.symmetric``)."""
    rows = np.asarray(rows, dtype=np.int64)
    cols = np.asarray(cols, dtype=np.int64)
    off = rows != cols
    isdir = np.zeros(n, dtype=bool)
    isdir[rows[~off]] = True
    isdir[rows[off]] = False
    keep = ~isdir[rows] & ~isdir[cols]
    r, c = rows[keep], cols[keep]
    for v in np.atleast_2d(vals):
        A = sp.csr_matrix((np.asarray(v)[keep], (r, c)), shape=(n, n))
        amax = abs(A).max() if A.nnz else 0.0
        if amax > 0 and abs(A - A.T).max() > rtol * amax:
            return False
    return True


class _LaneThread:
    """One solver lane's host thread: the lane's launches are issued here while the caller's thread issues lane 0's
    (the C calls release the GIL).  A queue pair instead of a ThreadPoolExecutor: submit is one C-level put (the
    executor's submit took ~15 us of the step-to-step turnaround before lane 0's first launch)."""

    def __init__(self):
        import queue
        import threading
        self._in, self._out = queue.SimpleQueue(), queue.SimpleQueue()
        self._th = threading.Thread(target=_LaneThread._loop, args=(self._in, self._out), name="pfr-lane",
                                    daemon=True)
        self._th.start()
        # the thread holds the queues only: an engine dropped without close() ends its lane threads
        weakref.finalize(self, self._in.put, None)

    @staticmethod
    def _loop(qin, qout):
        while True:
            item = qin.get()
            if item is None:
                return
            fn, arg = item
            try:
                fn(arg)
                qout.put(None)
            except BaseException as e:       # noqa: BLE001 -- handed to the caller's result()
                qout.put(e)
            del fn, arg, item

    def submit(self, fn, arg):
        self._in.put((fn, arg))

    def result(self):
        """The exception the submitted call raised, or None; waits for it."""
        return self._out.get()

    def close(self):
        self._in.put(None)
        self._th.join()


class _Engine:
    """Device state of one Problem: symbolic analysis, operator data and ``lanes``
    solvers, each with its own workspace and HIP stream.  A sweep splits its
    frequencies into one contiguous block per lane and runs the lanes
    concurrently; their kernels share the CUs (measured at C3: 2 lanes x 2,048
    frequencies 4 % faster than 1 lane x 4,096, 3-4 lanes slower)."""

    def __init__(self, prob: "Problem", device, n_freqs: int, max_batch: int | None, lanes: int | None = None,
                 symmetric: bool | None = None):
        self.device = device
        mats = prob.mats
        # structural pattern of the matrices that can be non-zero: for a mid-plane
        # symmetric material the B coefficients are identically zero, the KB
        # entries carry exact zeros and are dropped from the factorised pattern.
        active = [k for k in range(26) if not (prob.material.is_mps and KB_SLICE.start <= k < KB_SLICE.stop)]
        # entries that are exactly zero in every active matrix (explicit zeros of the FE layout)
        # are left out too: they change nothing, and with them out the Dirichlet rows hold
        # only their diagonal entry
        keep = prob.present[active].any(axis=0) & (mats[active] != 0).any(axis=0)
        self.keep = np.nonzero(keep)[0]
        rows, cols = prob.rows[self.keep], prob.cols[self.keep]
        n = prob.mat_size
        colptr = np.zeros(n + 1, dtype=np.int64)
        np.add.at(colptr, cols.astype(np.int64) + 1, 1)
        colptr = np.cumsum(colptr).astype(np.int32)
        vals = mats[:, self.keep]
        if symmetric is None:
            symmetric = os.environ.get("PFR_SYMMETRIC", "1") != "0"
        # symmetric mode when every matrix is complex symmetric away from the Dirichlet rows
        # (checked on the values): only L is formed, U = diag(U) L^T
        self.symmetric = bool(symmetric) and decoupled_symmetric(rows, cols, vals, n)
        # tuning knobs of the symbolic analysis (defaults in include/pfr.h): PFR_LEAF_SIZE,
        # PFR_RELAX="small,mid,big[,zmid,zbig]" (supernode amalgamation pivot limits and zero fractions), PFR_MAX_NS,
        # PFR_MD_DELTA, PFR_ORDERING (2: the exact-minimum-degree leaves of rounds 1-3, for A/B runs)
        env = lambda k: os.environ.get(k)  # noqa: E731
        self._sym_args = (n, colptr, rows.astype(np.int32))
        self._sym_kw = dict(symmetric=self.symmetric, ordering=int(env("PFR_ORDERING") or 0),
                            relax=tuple(float(v) for v in env("PFR_RELAX").split(",")) if env("PFR_RELAX") else None,
                            max_ns=int(env("PFR_MAX_NS")) if env("PFR_MAX_NS") else None,
                            md_delta=int(env("PFR_MD_DELTA")) if env("PFR_MD_DELTA") else None)
        self._leaf_env = int(env("PFR_LEAF_SIZE")) if env("PFR_LEAF_SIZE") else None
        self._syms = {}
        self._use_symbolic(n_freqs)
        self._lanes_req = int(os.environ.get("PFR_LANES", "2")) if lanes is None else int(lanes)
        self._lane_freqs = max(64, int(os.environ.get("PFR_LANE_FREQS", "256")))   # frequencies per lane at least
        self._fixed_batch = max_batch
        self.solvers, self.streams, self._pool = [], [], None
        self._spin_wait = os.environ.get("PFR_STEP_WAIT", "spin") != "block"
        self.n_lanes = 0
        self._seeded = False
        self._sized_for = set()
        # the coefficient matrices contracted for the gradient: all 18, or the 12 of A and D when the
        # coupling coefficients B vanish identically (mid-plane symmetric materials: dB/dtheta = 0, so
        # their gradient partials are exactly zero and need not be formed)
        self.kidx = np.r_[0:6, 12:18] if prob.material.is_mps else np.arange(18)
        self.n_stiff = int(self.kidx.size)
        self.stiff = torch.as_tensor(np.ascontiguousarray(vals[self.kidx].T), device=device)  # (nnz, n_stiff)
        I0, I0c, I2, I2c = prob.I0, prob.I0Corr, prob.I2, prob.I2Corr
        mass = I0 * (vals[18] + vals[20] + vals[22]) + I0c * (vals[19] + vals[21] + vals[23]) \
            + I2 * vals[24] + I2c * vals[25]                                                  # Problem.py:441-443
        self.mass = torch.as_tensor(np.ascontiguousarray(mass), device=device)
        self.mass_sum = I0 + I0c + I2 + I2c
        self.K = torch.empty(self.keep.size, dtype=torch.complex128, device=device)
        self.e = np.concatenate([np.zeros(12), RHS_WEIGHTS_D])
        aU, aV, aW = prob.averaging_vectors()
        self._sup = np.nonzero((aU != 0) | (aV != 0) | (aW != 0))[0]
        self._a3 = np.stack([aU[self._sup], aV[self._sup], aW[self._sup]])
        self._ts = prob.accelerometer.transverse_sensitivity
        self.rhs = prob.vec
        self._coef_key = None
        self.last_berr = None          # (F, 2) componentwise backward errors of the last sweep (device; a loss
                                       # step's buffer is reused -- overwritten -- by the next loss step)
        self.last_flags = None         # its status flags (host)
        # backward-error checks of every solve (pfr_set_check) and the functional correction (fr to
        # second order in the solve's error, the accuracy of the reference's refined UMFPACK solves) by
        # default; PFR_CHECK=<PFR_CHECK_* bits> / PFR_CHECK_TOL override; refinement (bits 4, 16) off by default
        self.check_mode = int(os.environ.get("PFR_CHECK", str(_native.PFR_CHECK_FORWARD | _native.PFR_CHECK_ADJOINT
                                                              | _native.PFR_CHECK_CORRECT)))
        self.check_tol = float(os.environ.get("PFR_CHECK_TOL", "1e-10"))
        # the selective adjoint refinement's group threshold (first-order fr error estimate)
        self.refine_tol = float(os.environ.get("PFR_REFINE_TOL", "2e-8"))
        self.ensure(n_freqs)

    def leaf_size_for(self, n_freqs: int) -> int:
        """Nested-dissection leaf size of the ordering for a sweep of ``n_freqs`` frequencies (DESIGN.md
        section 8, round 3).  Parts of at most this many nodes are ordered by multiple minimum degree:
        10,000 (one dissection at C3) gives the least fill and Schur-complement traffic but a deep tree
        (38 levels), whose per-level chains cost nothing when each level has thousands of workgroups
        and dominate the sparse solve passes of narrow sweeps; those get the shallower trees of more
        dissection levels.  C3, freq-solves/s at leaf 96 / 500 / 3,000 / 10,000 (late round 3, with the
        functional from the bottom-up passes): 512 frequencies 32.7k / 33.0k / 31.3k / 30.5k, 1,024
        41.1k / 42.8k / 43.5k / 44.0k, 2,048 - / 49.8k / 51.4k / 52.7k.  Round 4 (current kernels, alternated
        runs, profiles/r04/experiments/leaf*.txt): 512 frequencies leaf 96 / 150 / 200 / 250 / 300: 32.2-33.4k /
        34.2k / 34.9-35.1k / 33.4k / 33.3-33.9k; 1,024 leaf 600 / 1,000 / 2,000 / 10,000: 43.2k / 45.8-46.1k / 46.7k /
        44.5-44.9k; 2,048 leaf 1,000 / 2,000 / 10,000: 53.0k / 55.2k / 55.4-55.8k; 4,096: 10,000 best.  Round 5, with
        512 frequencies on two lanes of 256: leaf 120 / 200 / 350 / 700 / 1,000 / 2,000 / 5,000 / 10,000: 36.1-36.2k /
        36.8-37.0k / 36.7-37.2k / 36.8-36.9k / 37.9-38.4k / 36.2-38.0k / 38.1-38.3k / 33.5k; 1,024 leaf 1,000 / 2,000 /
        5,000 / 10,000: 48.4-48.6k / 50.3-50.4k / 50.2-50.8k / 48.5k; 2,048: 5,000 = 10,000 (gpurun_out/r6_leaf*).
        Round 6, C4's rank block (tools/ab_proxy.sh, 7 alternations on two boxes): leaf 600 / 1,000 / 2,000 / 3,000
        40.7-41.7k / 41.3-42.9k / 41.5-43.4k / 40.6-41.2k, 2,000 ahead of 1,000 in 6 of 7 pairs (+0.8 %;
        gpurun_out/lf_p512, lf2_p512): 2,000 for up to 512 frequencies."""
        if self._leaf_env is not None:
            return self._leaf_env
        n_freqs = max(1, n_freqs)
        return 200 if n_freqs <= 256 else 2000 if n_freqs <= 1024 else 10000

    def _use_symbolic(self, n_freqs: int) -> bool:
        """Select (building once) the symbolic analysis for a sweep width; True if it changed."""
        leaf = self.leaf_size_for(n_freqs)
        if leaf not in self._syms:
            self._syms[leaf] = _native.Symbolic(*self._sym_args, leaf_size=leaf, **self._sym_kw)
        changed = getattr(self, "sym", None) is not self._syms[leaf]
        self.sym = self._syms[leaf]
        self.stats = self.sym.stats()
        return changed

    def _lanes_for(self, n_freqs: int) -> int:
        """Solver lanes for a sweep of ``n_freqs``: a lane per PFR_LANE_FREQS (256) frequencies at most.  Round 3
        kept 512 frequencies on one lane (27.1k against 26.4k freq-solves/s with two); with round 5's kernels two
        lanes of 256 overlap each other's narrow-level chains and kernel drains: 36.2-36.8k -> 36.6-37.6k over five
        alternations, four lanes of 128 27.5k (profiles/EXPERIMENTS.md, round 5).  Round 6, C4's rank block
        (tools/strong_proxy.py --one 512, three alternations): two lanes of 256 41.5-41.6k, one lane of 512
        40.6-40.7k (gpurun_out/r6u); 512 frequencies spread over the band favoured one lane (41.7-41.8k against
        41.1-41.2k, gpurun_out/r6k_e512) -- the rank block is the C4 workload."""
        return max(1, min(self._lanes_req, -(-max(1, n_freqs) // self._lane_freqs)))

    def _shape_for(self, n_freqs: int):
        """(lanes, frequencies per chunk) for a sweep of ``n_freqs``: up to ``lanes`` lanes of at
        least 64 frequencies; per lane as many frequencies per chunk as fit in its share of ~85 %
        of the free HBM (multiple of 64, <= 4096), in even chunks."""
        n_freqs = max(1, n_freqs)
        n_lanes = self._lanes_for(n_freqs)
        if self._fixed_batch:
            return n_lanes, int(self._fixed_batch)
        per_lane = -(-n_freqs // n_lanes)
        free, _ = torch.cuda.mem_get_info(self.device)
        n = self._sym_args[0]
        # ours, if rebuilt: the workspaces, and the refinement's seed vectors the solvers already hold
        free += sum(self.sym.workspace_bytes(sv.max_batch) + (n * sv.max_batch * 16 if self._seeded else 0)
                    for sv in self.solvers)
        per64 = self.sym.workspace_bytes(64)
        if getattr(self, "check_mode", 0) & _native.PFR_CHECK_REFINE_ADJ:
            per64 += n * 64 * 16     # the refinement's fr seed vector (n x Fc), allocated on first use
        cap = max(64, min(4096, int(0.85 * free / n_lanes / per64) * 64))
        n_chunks = -(-per_lane // cap)
        return n_lanes, (-(-per_lane // n_chunks) + 63) // 64 * 64

    def ensure(self, n_freqs: int, refit: bool = False):
        """Size the lanes for a sweep of ``n_freqs`` frequencies.  The solvers are rebuilt only when
        the sweep needs more lanes or larger chunks than the current ones have (a small first call
        must not pin 1 lane and 64-frequency chunks on every later large sweep); smaller sweeps run
        on the existing solvers -- with their lanes and their ordering: the widest sweep so far fixes the
        elimination tree (a C4 rank, whose engine is first sized for its 512-frequency share, gets the
        shallow narrow-sweep tree; a 512-frequency sweep after a 4,096-frequency one runs on the deep
        tree, correct but slower)."""
        if self.solvers and not refit:
            per_lane = -(-max(1, n_freqs) // self.n_lanes)
            if n_freqs in self._sized_for or (self._lanes_for(n_freqs) <= self.n_lanes and per_lane <= self.max_batch):
                return
        self._sized_for.add(n_freqs)
        old = self.sym
        if self.solvers:
            self._use_symbolic(n_freqs)   # a rebuild for a wider sweep may take a deeper ordering
        lanes, batch = self._shape_for(n_freqs)
        if refit:
            # re-sized for what now has to fit beside the workspaces (set_check adding the refinement's seed
            # vectors): smaller chunks only when the current ones no longer fit
            if self.solvers and batch >= self.max_batch:
                return
            lanes = max(lanes, self.n_lanes)
        else:
            if self.solvers and lanes <= self.n_lanes and batch <= self.max_batch and self.sym is old:
                return
            lanes = max(lanes, self.n_lanes)
            batch = max(batch, self.max_batch if self.solvers else 0)
        if self.solvers:
            torch.cuda.synchronize(self.device)
        self.solvers, self.streams = [], []       # free the old workspaces before allocating
        if self._pool is not None:
            for t in self._pool:
                t.close()
            self._pool = None
        self.n_lanes = lanes
        self.solvers = [_native.Solver(self.sym, self.device.index, batch) for _ in range(lanes)]
        self._seeded = False           # no refinement seed vector allocated in the new solvers yet
        self.streams = [torch.cuda.Stream(self.device) for i in range(lanes)]
        if lanes > 1 and os.environ.get("PFR_PAR_LAUNCH", "1") != "0":
            self._pool = [_LaneThread() for _ in range(lanes - 1)]
        for sv in self.solvers:
            sv.set_stiffness(self.stiff, self.e[self.kidx])
            sv.set_operator(torch.view_as_real(self.K), self.mass)      # K(theta) shared by the lanes
            sv.set_functional(self._sup, self._a3, self._ts)
            sv.set_check(self.check_mode, self.check_tol)
            sv.set_refine_tol(self.refine_tol)
        self._coef_key = None          # new solvers: rhs scale not set yet

    def set_check(self, mode: int | None = None, tol: float | None = None):
        """Backward-error check mode (PFR_CHECK_* bits) and flag tolerance of every lane.  Turning on the
        selective adjoint refinement (PFR_CHECK_REFINE_ADJ) re-sizes the chunks when its seed vectors (n x chunk
        per lane, allocated on first use) would not fit beside the current workspaces."""
        adds_refine = mode is not None and bool(int(mode) & _native.PFR_CHECK_REFINE_ADJ) \
            and not (self.check_mode & _native.PFR_CHECK_REFINE_ADJ)
        if mode is not None:
            self.check_mode = int(mode)
        if tol is not None:
            self.check_tol = float(tol)
        for sv in self.solvers:
            sv.set_check(self.check_mode, self.check_tol)
        if adds_refine and self.solvers:
            self.ensure(max(self._sized_for) if self._sized_for else self.n_lanes * self.max_batch, refit=True)

    @property
    def solver(self):
        return self.solvers[0]

    @property
    def max_batch(self) -> int:
        return self.solver.max_batch

    def expand(self, v: torch.Tensor) -> torch.Tensor:
        """Partials over the contracted matrices (last axis n_stiff) -> over all 18 (zeros elsewhere)."""
        if self.n_stiff == 18:
            return v
        out = torch.zeros(v.shape[:-1] + (18,), dtype=v.dtype, device=v.device)
        # the index on the device once: a per-call host->device copy of it blocked the host until the
        # sweep had finished, so the small kernels after the sweep were only enqueued then
        key = str(v.device)
        if getattr(self, "_kidx_dev", (None, None))[0] != key:
            self._kidx_dev = (key, torch.as_tensor(self.kidx, device=v.device))
        out[..., self._kidx_dev[1]] = v
        return out

    def set_coefficients(self, c: np.ndarray):
        """Precombine K(theta) = sum_k c_k S_k on the device and the rhs scale."""
        key = c.tobytes()
        if key == self._coef_key:
            return
        self.solver.combine(np.asarray(c)[self.kidx], torch.view_as_real(self.K))
        beta = complex(self.e @ c)
        for sv in self.solvers:
            sv.set_rhs(self.rhs, beta, self.mass_sum)
        self._coef_key = key

    def _split(self, n):
        """Contiguous frequency block of each lane (multiples of 64 but the last)."""
        per = (-(-n // self.n_lanes) + 63) // 64 * 64
        return [(min(n, i * per), min(n, (i + 1) * per)) for i in range(self.n_lanes)]

    def _run(self, call, n, accum, lane_bufs=None, raw=False):
        """``call(solver, lo, hi, bufs)`` on every lane's stream; per-lane ``accum``
        buffers (zeros like each given tensor) are summed into the given tensors -- or, with
        ``lane_bufs`` (the caller's zeroed per-lane buffers, one list per lane), accumulated there and
        left to the caller.  With several lanes each lane's launches are issued from its own host
        thread (the C calls release the GIL): issued one after the other, the second lane started a
        whole sweep's enqueue time (~9 ms) after the first and finished that much later.  ``raw``: ``call`` issues
        native work only and takes the lane's stream handle as a fifth argument (no torch device / stream context
        per lane on the step's critical path)."""
        cur = torch.cuda.current_stream(self.device)
        jobs = []
        spans = [(i, sv, st, lo, hi) for i, (sv, st, (lo, hi)) in
                 enumerate(zip(self.solvers, self.streams, self._split(n))) if hi > lo]
        # the lanes ordered after the current stream and it after them by pfr_stream_order (one C call each;
        # Stream.wait_stream makes and destroys an event per call: host time before the first launch)
        cur_h = cur.cuda_stream
        for i, sv, st, lo, hi in spans:
            # the lane's accumulation buffers are zero-filled on the current stream BEFORE the lane
            # stream is ordered after it (k_reduce accumulates into them with +=); one lane accumulates
            # straight into the given tensors
            if lane_bufs is not None:
                bufs = lane_bufs[i]
            else:
                bufs = list(accum) if len(spans) == 1 else [None if a is None else torch.zeros_like(a) for a in accum]
            _native.stream_order(st.cuda_stream, cur_h)
            jobs.append((i, sv, st, lo, hi, bufs))
        if _HT is not None:
            _HT("lanes_ordered")

        def lane(job):
            _, sv, st, lo, hi, bufs = job
            if raw:
                call(sv, lo, hi, bufs, st.cuda_stream)
                return
            with torch.cuda.device(self.device), torch.cuda.stream(st):
                call(sv, lo, hi, bufs)

        err = None
        if len(jobs) > 1 and self._pool is not None:
            # lanes 1.. on their threads, lane 0 on this thread meanwhile (one thread handoff less before the
            # first launch: the GPU idles from the previous step's result until then)
            for t, j in zip(self._pool, jobs[1:]):
                t.submit(lane, j)
            if _HT is not None:
                _HT("submitted")
            try:
                lane(jobs[0])
            except Exception as e:           # noqa: BLE001 -- re-raised once every lane is joined
                err = e
            errs = [t.result() for t, _ in zip(self._pool, jobs[1:])]   # every lane has issued its work (or failed) ...
            errs = [e for e in errs if e is not None]
            err = err if err is not None else (errs[0] if errs else None)
        else:
            for j in jobs:
                try:
                    lane(j)
                except Exception as e:       # noqa: BLE001 -- re-raised once every lane is joined
                    err = e
                    break
        for i, _, st, _, _, bufs in jobs:    # ... and the current stream is ordered after all of them
            _native.stream_order(cur_h, st.cuda_stream)
            for b in bufs:
                if b is not None:
                    b.record_stream(cur)
        if err is not None:
            raise err
        if lane_bufs is not None:
            return
        for _, _, st, _, _, bufs in jobs:
            for a, b in zip(accum, bufs):
                if a is not None and b is not a:
                    a.add_(b)

    def loss_step(self, freqs, loss_type, ref, scale):
        """One loss + gradient sweep with the step buffers reused across calls (the optimiser / bench loop:
        the host's step-to-step turnaround is GPU idle time).  Per lane, loss and the contracted partials
        accumulate into one slot of a single device buffer whose last entry receives the number of flagged
        frequencies; one fill per buffer, one device->host copy.  Returns (loss sum, w (18,) complex, flags
        device tensor, flagged count); the backward errors land in ``last_berr``."""
        n = freqs.numel()
        key = (n, self.n_lanes, id(self.solvers[0]))
        b = self._step_bufs.get(key) if hasattr(self, "_step_bufs") else None
        L, m = self.n_lanes, 2 + 2 * self.n_stiff
        if b is None:
            # the lanes' loss / w slots (float64) and the flags (int32) in one device buffer: one device->host
            # copy per step, the flagged count taken on the host (no count kernels after the sweep)
            raw = torch.empty(8 * L * m + 4 * n, dtype=torch.uint8, device=self.device)
            acc = raw[:8 * L * m].view(torch.float64)
            lanes = [[acc[l * m:l * m + 1], acc[l * m + 2:(l + 1) * m].view(self.n_stiff, 2)] for l in range(L)]
            b = (acc, lanes, raw[8 * L * m:].view(torch.int32),
                 torch.empty((n, 2), dtype=torch.float64, device=self.device), raw,
                 torch.empty(raw.numel(), dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
            self._step_bufs = {key: b}            # one shape at a time (a new size replaces it)
        acc, lanes, flags, berr, raw, host, done = b
        # no fills here: every lane's sweep initialises its loss / w slots, flags and backward errors in its first
        # kernel (pfr_sweep_fresh)
        # the lanes' views of this step's tensors, made once per (buffers, freqs, ref): slicing costs host time
        # on the step-to-step turnaround
        vkey = (key, freqs.data_ptr(), ref.data_ptr(), freqs.numel())
        views = self._step_views.get(vkey) if hasattr(self, "_step_views") else None
        if views is None:
            views = {lo: (berr[lo:hi], freqs[lo:hi], ref[lo:hi], flags[lo:hi]) for lo, hi in self._split(n)}
            ran = [hi > lo for lo, hi in self._split(n)]
            views["_act"] = None if all(ran) else np.nonzero(ran)[0]
            self._step_views = {vkey: views}

        def call(sv, lo, hi, bufs, stream):
            vb, vf, vr, vfl = views[lo]
            sv.set_check(self.check_mode, self.check_tol, vb)
            try:
                sv.sweep(vf, loss_type, ref=vr, scale=scale, loss=bufs[0], w=bufs[1], flags=vfl, fresh=True,
                         stream=stream)
            finally:
                sv.set_check(self.check_mode, self.check_tol)
        if self.check_mode & _native.PFR_CHECK_REFINE_ADJ:
            self._seeded = True
        self._run(call, n, None, lane_bufs=lanes, raw=True)
        # the result into pinned memory and the host polling for it: a blocking copy returned ~85 us after the copy
        # had finished on the GPU (the host thread woken from its sleep, gpurun_out/tl/timeline.txt) -- GPU idle
        # before the next step's first launch.  PFR_STEP_WAIT=block: the blocking copy.
        if self._spin_wait:
            host.copy_(raw, non_blocking=True)
            done.record(torch.cuda.current_stream(self.device))
            while not done.query():
                pass
            if _HT is not None:
                _HT("copy_done")
            hb = host.numpy()
        else:
            hb = raw.cpu().numpy()
        h = hb[:8 * L * m].view(np.float64).reshape(L, m)
        self.last_flags_host = hb[8 * L * m:].view(np.int32).copy()
        # summed over the lanes that swept (a lane with no frequencies ran nothing: its slot was never initialised);
        # a lane's slot: loss, (unused), then its n_stiff partials as complex pairs
        act = views["_act"]
        tot = h[act].sum(axis=0) if act is not None else h.sum(axis=0)
        wk = tot[2:].view(np.complex128)
        if wk.size == 18:
            w = wk.copy()
        else:
            w = np.zeros(18, dtype=np.complex128)
            w[self.kidx] = wk
        self.last_berr = berr
        return float(tot[0]), w, flags, int(np.count_nonzero(self.last_flags_host))

    def sweep(self, freqs, loss_type=_native.LOSS_NONE, ref=None, scale=1.0, fr=None, loss=None, w=None,
              flags=None, berr=None):
        """``Solver.sweep`` over all lanes (fr / flags / berr (F, 2) written in place, loss / w
        accumulated)."""
        if self.check_mode & _native.PFR_CHECK_REFINE_ADJ:
            self._seeded = True        # the lanes allocate their refinement seed vectors in this sweep

        def call(sv, lo, hi, bufs):
            if berr is not None:
                sv.set_check(self.check_mode, self.check_tol, berr[lo:hi])
            try:
                sv.sweep(freqs[lo:hi], loss_type, ref=None if ref is None else ref[lo:hi], scale=scale,
                         fr=None if fr is None else fr[lo:hi], loss=bufs[0], w=bufs[1],
                         flags=None if flags is None else flags[lo:hi])
            finally:
                if berr is not None:
                    sv.set_check(self.check_mode, self.check_tol)
        self._run(call, freqs.numel(), [loss, w])

    def hessian_sweep(self, freqs, loss_type, ref, scale, dcoef, loss=None, w=None, h=None, flags=None):
        def call(sv, lo, hi, bufs):
            sv.hessian_sweep(freqs[lo:hi], loss_type, ref[lo:hi], scale, dcoef, loss=bufs[0], w=bufs[1],
                             h=bufs[2], flags=None if flags is None else flags[lo:hi])
        self._run(call, freqs.numel(), [loss, w, h])

    # ---- measurement (bench.py)
    def set_timing(self, on, kernels=False):
        for sv in self.solvers:
            sv.set_timing(on, kernels)

    def last_timings(self) -> np.ndarray:
        """Per-phase device ms of the last call, summed over the lanes (lanes overlap in time)."""
        return sum(sv.last_timings() for sv in self.solvers)

    def last_kernel_timings(self):
        ms, n = zip(*(sv.last_kernel_timings() for sv in self.solvers))
        return sum(ms), sum(n)


_JET_TYPES = ('isotropic', 'orthotropic', 'orthotropic_d4', 'sol', 'symm_sol')
_HT = None          # host-turnaround marks (tools/host_turnaround.py sets a callable; None in use)


def _coeffs18(transform, params: torch.Tensor) -> torch.Tensor:
    A, B, D = transform(params)
    return torch.cat([A, B, D]).to(torch.complex128)


class _SweepFR(torch.autograd.Function):
    """fr(c) for a frequency vector; backward = adjoint sweep with dL/dfr."""

    @staticmethod
    def forward(ctx, c, engine, freqs):
        cn = c.detach().cpu().numpy()
        engine.set_coefficients(cn)
        fr = torch.empty(freqs.numel(), dtype=torch.float64, device=engine.device)
        flags = torch.zeros(freqs.numel(), dtype=torch.int32, device=engine.device)
        berr = torch.full((freqs.numel(), 2), float('nan'), dtype=torch.float64, device=engine.device)
        engine.sweep(freqs, _native.LOSS_NONE, fr=fr, flags=flags, berr=berr)
        engine.last_berr = berr
        engine.last_flags = _check_flags(flags)
        ctx.engine, ctx.freqs, ctx.cn = engine, freqs, cn
        return fr

    @staticmethod
    def backward(ctx, grad_fr):
        engine = ctx.engine
        engine.set_coefficients(ctx.cn)
        ref = torch.zeros(ctx.freqs.numel(), dtype=torch.complex128, device=engine.device)
        ref.real.copy_(grad_fr.to(torch.float64))
        w = torch.zeros(engine.n_stiff, dtype=torch.complex128, device=engine.device)
        loss = torch.zeros(1, dtype=torch.float64, device=engine.device)
        # the cotangent sweep's solves are checked like the forward ones: flags and backward errors
        # reported, not dropped
        flags = torch.zeros(ctx.freqs.numel(), dtype=torch.int32, device=engine.device)
        berr = torch.full((ctx.freqs.numel(), 2), float('nan'), dtype=torch.float64, device=engine.device)
        engine.sweep(ctx.freqs, _native.LOSS_COTANGENT, ref=torch.view_as_real(ref), scale=1.0,
                     loss=loss, w=torch.view_as_real(w), flags=flags, berr=berr)
        engine.last_berr = berr
        engine.last_flags = _check_flags(flags)
        return torch.conj(engine.expand(w)).to(torch.complex128).cpu(), None, None


class _SweepLoss(torch.autograd.Function):
    """Fused loss + gradient: one factorisation per frequency (forward + adjoint)."""

    @staticmethod
    def forward(ctx, c, engine, freqs, ref, loss_id, n_total, reduce_fn):
        cn = c.detach().cpu().numpy()
        engine.set_coefficients(cn)
        if reduce_fn is None:
            # the single-process step: reused buffers, one device->host copy (_Engine.loss_step)
            lsum, w, flags, nflag = engine.loss_step(freqs, loss_id, torch.view_as_real(ref), 1.0 / n_total)
            engine.last_flags = _check_flags(flags) if nflag else np.zeros(flags.numel(), np.int32)
            ctx.save_for_backward(torch.from_numpy(w))
            return torch.tensor(lsum / n_total, dtype=torch.float64)
        w = torch.zeros(engine.n_stiff, dtype=torch.complex128, device=engine.device)
        loss = torch.zeros(1, dtype=torch.float64, device=engine.device)
        flags = torch.zeros(freqs.numel(), dtype=torch.int32, device=engine.device)
        berr = torch.full((freqs.numel(), 2), float('nan'), dtype=torch.float64, device=engine.device)
        engine.sweep(freqs, loss_id, ref=torch.view_as_real(ref), scale=1.0 / n_total,
                     loss=loss, w=torch.view_as_real(w), flags=flags, berr=berr)
        engine.last_berr = berr
        packed = torch.cat([loss.to(torch.complex128), engine.expand(w)])
        if reduce_fn is not None:
            packed = reduce_fn(packed)
        # one device->host copy per step: loss, gradient partials and the number of flagged frequencies
        # (the flags themselves are copied only when some are set)
        host = torch.cat([packed, torch.count_nonzero(flags).to(torch.complex128).reshape(1)]).cpu()
        engine.last_flags = _check_flags(flags) if host[-1].real != 0 else np.zeros(flags.numel(), np.int32)
        ctx.save_for_backward(host[1:-1])
        return host[0].real / n_total

    @staticmethod
    def backward(ctx, g):
        (w,) = ctx.saved_tensors
        return torch.conj(w) * g, None, None, None, None, None, None


class _JetSweepLoss(torch.autograd.Function):
    """params -> loss as ONE autograd node for the material types of the jet transform (_abd_jet.py): c(theta) and
    its Jacobian J from the jet pass, loss and the partials w from the fused sweep (_Engine.loss_step), and
    dL/dtheta = Re(w J) -- the product _Coeffs.backward forms from _SweepLoss.backward's conj(w) -- already in the
    forward, so that the backward is one scale.  The same values, bit for bit, as the chain
    params.to(float64).cpu() * scaling -> _Coeffs -> _SweepLoss, with three autograd nodes fewer on the host's
    step-to-step turnaround (the GPU idles from one step's result to the next step's first launch)."""

    @staticmethod
    def forward(ctx, params, material, h, scaling, engine, freqs, ref, loss_id, n_total):
        # scaling: 1.0 or a float64 numpy array (the host arithmetic in numpy: the same IEEE products as the
        # chain's torch ones, a few us less per step)
        ctx.cast = params.dtype != torch.float64 or params.device.type != "cpu"
        p = (params.detach().to(torch.float64).cpu() if ctx.cast else params.detach()).numpy() * scaling
        c, J = _cached_abd(material, h, p)
        engine.set_coefficients(c)
        lsum, w, flags, nflag = engine.loss_step(freqs, loss_id, torch.view_as_real(ref), 1.0 / n_total)
        engine.last_flags = _check_flags(flags) if nflag else np.zeros(flags.numel(), np.int32)
        # dL/dparams for an incoming gradient of 1 (the chain's values for it, bit for bit: Re(w J) * scaling)
        ctx.gt = torch.from_numpy(np.real(w @ J) * scaling)
        ctx.dtype, ctx.device = params.dtype, params.device
        return torch.scalar_tensor(lsum / n_total, dtype=torch.float64)

    @staticmethod
    def backward(ctx, g):
        grad = ctx.gt * g
        return (grad.to(dtype=ctx.dtype, device=ctx.device) if ctx.cast else grad), None, None, None, None, None, \
            None, None, None


def _check_flags(flags):
    """Warn about frequencies whose solves were flagged (one device->host copy of F int32)."""
    f = flags.cpu().numpy()
    if not f.any():
        return f
    msgs = []
    for bit, what in ((_native.PFR_FLAG_BAD_PIVOT, "hit a zero/non-finite static pivot"),
                      (_native.PFR_FLAG_BACKWARD_ERROR, "have a forward solution whose backward error exceeds "
                                                        "the check tolerance"),
                      (_native.PFR_FLAG_BACKWARD_ERROR_ADJ, "have an adjoint solution whose backward error exceeds "
                                                            "the check tolerance")):
        n = int(np.count_nonzero(f & bit))
        if n:
            msgs.append(f"{n} frequencies {what}")
    warnings.warn("; ".join(msgs) + " -- their results are not reliable (Problem.solveForwardChecked reports "
                  "the backward errors; PFR_CHECK=15 adds a refinement step)", RuntimeWarning)
    return f


class Problem:
    """Geometry + known parameters; builds the FE system once, exposes differentiable FR/loss."""

    def __init__(self, geometry: Geometry = None, material: Material = None, accel: Accelerometer = None,
                 ref_fr: tuple = None, *, cpu: int | None = 0, spath: str | os.PathLike = None,
                 device=None, max_batch: int | None = None):
        if (geometry, accel, material, spath) == (None,) * 4:                       # Problem.py:86-87
            raise ValueError('Cannot create a Problem object without arguments.')
        self.n_cpu = cpu
        self.geometry, self.material, self.accelerometer = geometry, material, accel
        if spath is None:
            if None in (geometry, accel, material):
                raise ValueError('Cannot create a Problem object without `spath` argument if any of '
                                 '`geometry`, `accel`, `material` arguments is `None`.')
        else:
            self._load_setup(spath, geometry, material, accel)
        if self.material.has_params:
            self.parameters = self.material.get_parameters()
        else:
            warnings.warn('Some elastic moduli of a material were not provided, solving forward problem as '
                          'standalone will not be possible.', RuntimeWarning)
        if ref_fr is not None:
            self.reference_fr = ref_fr
        self.e = self.geometry.height / 2.0
        self.rho = self.material.density
        self._device = device
        self._max_batch = max_batch
        self._engine = None
        self._fr_function = None
        self._build_system()

    # ------------------------------------------------------------------ setup
    def _load_setup(self, spath, geometry, material, accel):
        """``setup.json`` folder semantics of Problem.py:102-214."""
        if not isinstance(spath, (str, os.PathLike)):
            raise TypeError(f'Argument `spath` should have one of the following types: str | os.PathLike, '
                            f'not {type(spath)}.')
        if not os.path.isabs(spath):
            spath = os.path.join(_PKG_DIR, 'setups', spath)
        if not os.path.exists(spath):
            raise ValueError(f'Path of the setup {spath} does not exist.')
        if not os.path.isdir(spath):
            raise ValueError(f'Selected path {spath} is not a directory.')
        fpath = os.path.join(spath, 'setup.json')
        if not os.path.exists(fpath):
            raise FileNotFoundError(f'`setup.json` file was not found in setup directory {spath}.')
        with open(fpath) as f:
            sp = json.load(f)
        if 'accelerometer' in sp:
            v = sp['accelerometer']
            if isinstance(v, str):
                self.accelerometer = Accelerometer(v)
            elif isinstance(v, dict):
                self.accelerometer = Accelerometer(AccelerometerParams(**v))
            else:
                raise TypeError(f'In file {fpath} key `accelerometer` should have a value with type `str` or `dict`.')
        if 'material' in sp:
            v = sp['material']
            if not isinstance(v, (str, dict)):
                raise TypeError(f'In file {fpath} key `material` should have a value with type `str` or `dict`.')
            self.material = get_material(v)
        if material is not None:
            self.material = material
        if accel is not None:
            self.accelerometer = accel
        if geometry is not None:
            self.geometry = geometry
        elif 'geometry' in sp:
            g = dict(sp['geometry'])
            if 'template' not in g:
                raise ValueError(f'Cannot create Geometry object, file {fpath} should contain `template` inside '
                                 '`geometry` (FreeFEM `edp` geometries need FreeFem++, not available).')
            templ = g.pop('template')
            ny = g.pop('ny', 6)
            self.geometry = Geometry(templ, accelerometer=self.accelerometer, params=GeometryParams(**g), ny=ny)
        freq_file = os.path.join(spath, 'freqs.npy')
        if os.path.exists(freq_file):
            freqs = np.load(freq_file)
            amp = np.load(os.path.join(spath, 'amp.npy'))
            ph = os.path.join(spath, 'phase.npy')
            phase = np.load(ph) if os.path.exists(ph) else np.zeros_like(amp)
            self.reference_fr = (freqs, amp * np.exp(1j * phase))
        if None in (self.accelerometer, self.geometry, self.material):
            raise RuntimeError('One of the `geometry`, `accelerometer`, `materials` attributes was not provided '
                               'in setup.json nor as an argument.')

    def _build_system(self):
        """FE matrices + union pattern + inertia constants (Problem.py:310-374)."""
        out = load_matrices_unsymm(self.geometry.build_varfs())
        mats = out[0]
        self.mat_size = mats[0].shape[0]
        up = union_pattern(mats)
        self.sparsity = up.nnz / self.mat_size ** 2
        self.rows, self.cols = up.rows, up.cols
        self.colptr, self.rowind = up.colptr, up.rowind
        self.mats = up.values                                   # (26, nnz), CSC order
        self.present = np.zeros_like(up.values, dtype=bool)
        n = self.mat_size
        keys = up.rows.astype(np.int64) + n * up.cols.astype(np.int64)
        for k, m in enumerate(mats):
            c = m.tocoo()
            self.present[k, np.searchsorted(keys, c.row.astype(np.int64) + n * c.col.astype(np.int64))] = True
        (self.vec, self.interp_mat, self.interp_mat_Lh, self.Lh_size, self.Mh_size, self.mesh,
         self.interp_mat_Wx, self.interp_mat_Wy) = out[1:]
        acc = self.accelerometer
        rho_corr = acc.mass / (np.pi * acc.radius ** 2) / acc.height if acc is not None else 0.0
        h = self.geometry.height
        self.I0 = h * self.rho                                                  # Problem.py:367-374
        self.I0Corr = acc.height * rho_corr
        self.I2 = self.rho * h ** 3 / 12
        self.I2Corr = rho_corr / 3 * ((h / 2 + acc.height) ** 3 - h ** 3 / 8)

    def averaging_vectors(self):
        """aU, aV, aW with U = aU . x etc.: ``mean(I @ x) = (1^T I / P) @ x`` (Problem.py:454-462)."""
        L, n = self.Lh_size, self.mat_size
        k = self.accelerometer.effective_height * self.accelerometer.height
        P = self.interp_mat_Lh.shape[0]
        aU, aV, aW = np.zeros(n), np.zeros(n), np.zeros(n)
        aU[:L] = self.interp_mat_Lh.sum(0) / P
        aU[2 * L:] = -k * self.interp_mat_Wx.sum(0) / P
        aV[L:2 * L] = self.interp_mat_Lh.sum(0) / P
        aV[2 * L:] = -k * self.interp_mat_Wy.sum(0) / P
        aW[2 * L:] = self.interp_mat.sum(0) / P
        return aU, aV, aW

    # ------------------------------------------------------------------ engine
    @property
    def device(self):
        if self._device is None:
            self._device = _default_device()
        return torch.device(self._device)

    def engine(self, n_freqs: int | None = None) -> _Engine:
        """The device engine, sized -- and re-sized when a sweep needs more -- for ``n_freqs``
        (``None``: as it is, or for 1024 frequencies when it is first built)."""
        if self._engine is None:
            dev = self.device
            if dev.type != 'cuda':
                raise _native.NativeError('the plate solver needs a ROCm device (no CPU fallback)')
            self._engine = _Engine(self, dev, 1024 if n_freqs is None else n_freqs, self._max_batch)
        elif n_freqs is not None:
            self._engine.ensure(n_freqs)
        return self._engine

    def _transform(self):
        return self.material.get_ABD_transform(self.geometry.height)

    def _coeffs(self, transform, p: torch.Tensor) -> torch.Tensor:
        """c(theta) (18 complex) differentiable in theta: the jet transform (value and Jacobian in one numpy
        pass, backward one product: _abd_jet.py) for the material types of Material.py, torch autograd
        through ``transform`` otherwise."""
        if self.material.atype in _JET_TYPES:
            return _jet_coeffs18(self.material, self.geometry.height, p)
        return _coeffs18(transform, p)

    def _freqs(self, freqs) -> torch.Tensor:
        return torch.as_tensor(np.asarray(freqs, dtype=np.float64) if not isinstance(freqs, torch.Tensor)
                               else freqs, dtype=torch.float64, device=self.device).contiguous()

    # ------------------------------------------------------------------ API
    def getFRFunction(self) -> Callable:
        """``fr(freqs, params) -> (F,) float64 tensor`` on the device, differentiable in params
        (``Problem.py:377-518``).  Cached per instance while the caller holds it (the reference's ``functools.cache`` on the
        method would keep every Problem -- and its device workspaces -- alive for the process)."""
        fn = self._fr_function() if self._fr_function is not None else None
        if fn is not None:
            return fn
        transform = self._transform()

        def fr_function(freqs, params):
            f = self._freqs(freqs)
            p = params if isinstance(params, torch.Tensor) else torch.as_tensor(np.asarray(params, dtype=np.float64))
            c = self._coeffs(transform, p.to(torch.float64).cpu())
            return _SweepFR.apply(c, self.engine(f.numel()), f)

        self._fr_function = weakref.ref(fr_function)    # no Problem <-> closure reference cycle
        return fr_function

    getAFCFunction = getFRFunction

    def solveForward(self, freqs, params=None, *, distributed: bool = False) -> np.ndarray:
        """Frequency response at ``freqs`` [Hz] (``Problem.py:611-639``).

        With ``distributed=True`` and an initialised ``torch.distributed`` group every rank sweeps
        its contiguous block of ``freqs`` and one all-gather assembles the whole response on every
        rank."""
        if params is None:
            params = self.parameters
        if distributed:
            from .distributed import all_gather_cat, shard_range
            f = np.asarray(freqs, dtype=np.float64)
            lo, hi = shard_range(f.size)
            with torch.no_grad():
                part = self.getFRFunction()(f[lo:hi], params) if hi > lo else \
                    torch.zeros(0, dtype=torch.float64, device=self.device)
                return all_gather_cat(part, f.size).cpu().numpy()
        with torch.no_grad():
            return self.getFRFunction()(freqs, params).cpu().numpy()

    solve_forward = solveForward

    def solveForwardChecked(self, freqs, params=None, *, refine: bool = False, correct: bool | None = None):
        """``(fr, berr, flags)``: the forward sweep with the componentwise backward error of every
        frequency's solve (``max_i |b - A x|_i / (|A||x| + |b|)_i``, the measure UMFPACK's
        refinement monitors) and its status flags (PFR_FLAG_*); ``refine=True`` adds one step of
        iterative refinement on the same factors first (as the reference's UMFPACK solves do by
        default, ``InnerState.h:246-247`` with a NULL Control); ``correct`` turns the functional
        correction on / off (None: the engine's setting, on by default)."""
        if params is None:
            params = self.parameters
        f = self._freqs(freqs)
        p = torch.as_tensor(np.asarray(params, dtype=np.float64))
        c = _coeffs18(self._transform(), p).detach().numpy()
        eng = self.engine(f.numel())
        eng.set_coefficients(c)
        fr = torch.empty(f.numel(), dtype=torch.float64, device=eng.device)
        flags = torch.zeros(f.numel(), dtype=torch.int32, device=eng.device)
        berr = torch.full((f.numel(), 2), float('nan'), dtype=torch.float64, device=eng.device)
        mode = eng.check_mode
        m = mode | _native.PFR_CHECK_FORWARD | (_native.PFR_CHECK_REFINE if refine else 0)
        if correct is not None:
            m = (m | _native.PFR_CHECK_CORRECT) if correct else (m & ~_native.PFR_CHECK_CORRECT)
        eng.set_check(m)
        try:
            eng.sweep(f, _native.LOSS_NONE, fr=fr, flags=flags, berr=berr)
        finally:
            eng.set_check(mode)
        return fr.cpu().numpy(), berr[:, 0].cpu().numpy(), flags.cpu().numpy()

    def getLossFunction(self, frequencies, reference_fr, func_type: str, scaling_params=None,
                        *, distributed: bool = False) -> Callable:
        """``loss(params) -> 0-dim tensor`` (``Problem.py:933-980``).

        With ``distributed=True`` and an initialised ``torch.distributed`` group,
        every rank sweeps its contiguous block of the frequencies and one
        all-reduce combines loss and gradient partials.
        """
        frequencies = np.asarray(frequencies)
        reference_fr = np.asarray(reference_fr)
        assert frequencies.shape[0] == reference_fr.shape[0]
        if func_type not in _native.LOSS_IDS:
            raise ValueError(f'Function type "{func_type}" is not supported!')
        loss_id = _native.LOSS_IDS[func_type]
        scaling = 1.0 if scaling_params is None else torch.as_tensor(np.array(scaling_params, dtype=np.float64))
        scaling_np = 1.0 if scaling_params is None else np.array(scaling_params, dtype=np.float64)
        n_total = frequencies.shape[0]
        lo, hi, reduce_fn = 0, n_total, None
        if distributed:
            from .distributed import shard_range, all_reduce_sum
            lo, hi = shard_range(n_total)
            reduce_fn = all_reduce_sum
        transform = self._transform()
        f_local = self._freqs(frequencies[lo:hi])
        ref_local = torch.as_tensor(reference_fr[lo:hi].astype(np.complex128), device=self.device)

        def loss(params):
            p = params if isinstance(params, torch.Tensor) else torch.as_tensor(np.asarray(params, dtype=np.float64))
            if reduce_fn is None and self.material.atype in _JET_TYPES:
                # one autograd node (host turnaround of the optimiser / bench loop)
                return _JetSweepLoss.apply(p, self.material, self.geometry.height, scaling_np,
                                           self.engine(max(1, hi - lo)), f_local, ref_local, loss_id, n_total)
            c = self._coeffs(transform, p.to(torch.float64).cpu() * scaling)
            return _SweepLoss.apply(c, self.engine(max(1, hi - lo)), f_local, ref_local, loss_id, n_total, reduce_fn)

        return loss

    def getLossHessianFunction(self, frequencies, reference_fr, func_type: str, scaling_params=None,
                               *, distributed: bool = False) -> Callable:
        """``model(params) -> (loss, grad, hessian)`` (numpy) of ``getLossFunction``'s loss.

        Replaces the reference's forward-over-reverse Hessian (``jax.jacobian(grad)``,
        ``Optimizers.py:125-136``; its mode-4 solves refactorise per direction,
        ``InnerState.h:289-305``): one GPU sweep factors each frequency once and
        reuses the factors for the tangent solves ``A dx_i = db_i - dA_i x`` and the
        second-order adjoints ``A^T dl_i = dG_i - dA_i^T l`` of every parameter
        direction; the material transform's first and second derivatives come
        from torch autograd on the host.
        """
        frequencies = np.asarray(frequencies)
        reference_fr = np.asarray(reference_fr)
        assert frequencies.shape[0] == reference_fr.shape[0]
        if func_type not in ('MSE', 'RMSE', 'MSE_AFC', 'MSE_LOG_AFC'):
            raise ValueError(f'Function type "{func_type}" is not supported!')
        loss_id = _native.LOSS_IDS[func_type]
        scaling = 1.0 if scaling_params is None else torch.as_tensor(np.array(scaling_params, dtype=np.float64))
        n_total = frequencies.shape[0]
        lo, hi, reduce_fn = 0, n_total, None
        if distributed:
            from .distributed import shard_range, all_reduce_sum
            lo, hi = shard_range(n_total)
            reduce_fn = all_reduce_sum
        transform = self._transform()
        f_local = self._freqs(frequencies[lo:hi])
        ref_local = torch.as_tensor(reference_fr[lo:hi].astype(np.complex128), device=self.device)

        def c_real(p):
            return torch.view_as_real(_coeffs18(transform, p * scaling)).reshape(-1)      # (36,)

        def model(params):
            p = torch.as_tensor(np.asarray(params, dtype=np.float64)).detach()
            n = p.numel()
            if self.material.atype in _JET_TYPES:
                # the same c (to the bit) as getLossFunction's jet transform, and its Jacobian in p
                from ._abd_jet import abd_and_jacobian
                sc = np.broadcast_to(np.asarray(scaling, dtype=np.float64), (n,))
                c, J = abd_and_jacobian(self.material, self.geometry.height, (p * scaling).numpy())
                dc = J * sc[None, :]                                                      # (18, n)
            else:
                c = _coeffs18(transform, p * scaling).detach().numpy()
                jac = torch.autograd.functional.jacobian(c_real, p).numpy().reshape(18, 2, n)
                dc = jac[:, 0] + 1j * jac[:, 1]                                            # (18, n)
            d2 = np.stack([torch.autograd.functional.hessian(lambda x, m=m: c_real(x)[m], p).numpy()
                           for m in range(36)]).reshape(18, 2, n, n)
            d2c = d2[:, 0] + 1j * d2[:, 1]                                                 # (18, n, n)
            eng = self.engine(max(1, hi - lo))
            eng.set_coefficients(c)
            dev = eng.device
            w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
            h = torch.zeros(n, eng.n_stiff, dtype=torch.complex128, device=dev)
            loss = torch.zeros(1, dtype=torch.float64, device=dev)
            flags = torch.zeros(f_local.numel(), dtype=torch.int32, device=dev)
            eng.hessian_sweep(f_local, loss_id, torch.view_as_real(ref_local), 1.0 / n_total, dc[eng.kidx].T,
                              loss=loss, w=torch.view_as_real(w), h=torch.view_as_real(h), flags=flags)
            _check_flags(flags)
            packed = torch.cat([loss.to(torch.complex128), eng.expand(w), eng.expand(h).reshape(-1)])
            if reduce_fn is not None:
                packed = reduce_fn(packed)
            packed = packed.cpu().numpy()
            val = packed[0].real / n_total
            w_, h_ = packed[1:19], packed[19:].reshape(n, 18)
            grad = np.real(w_ @ dc)
            hess = np.real(h_ @ dc) + np.real(np.einsum('k,kij->ij', w_, d2c))
            return float(val), grad, 0.5 * (hess + hess.T)

        return model

    def solveInverse(self, *args, **kwargs):
        from .inverse import solve_inverse
        return solve_inverse(self, *args, **kwargs)

    def solveInverseLocal(self, *args, **kwargs):
        return self.solveInverse(*args, **kwargs)
