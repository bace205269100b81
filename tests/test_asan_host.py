"""Sanitizer run of the host C-ABI's planning code ("race detection / sanitizers"; the
reference builds with -Wall -g only, source/jax_plate_lib/CMakeLists.txt:6).

``make -C plate_inverse_problem_amd/csrc asan-host`` builds ``csrc/asan_driver.cpp`` + ``symbolic.cpp`` +
``plan.cpp`` -- the ``pfr::analyse`` that ``pfr_symbolic_create`` runs and the ``pfr::build_plan`` /
``pfr::workspace`` that ``pfr_solver_create`` runs (every record array the kernels gather through, the level
tables, the Dirichlet lists, the contraction entries, the chunk buffers' sizes) -- with g++
``-fsanitize=address,undefined`` (no recovery: any finding aborts the run with a non-zero status).  The driver
runs every ordering the engine and the tests use on the plate patterns (MMD and nested dissection at every leaf
size of the width rule, the exact-minimum-degree and natural orderings, general and symmetric analyses, the
support-last and max_ns options) up to the C3 mesh; the statistics must equal libpfr's for the same input, and
``pfr::check_plan`` must accept the plan of every engine shape (chunks of 64 .. 4,096 frequencies, Schur block
thresholds 0 / 4 / 24, frequency-major levels off / up to 4 fronts / all, solve split targets): every element id,
nz and record offset a launch takes from the plan inside the buffer it addresses, the per-workgroup partial
buffers sized for the grids that write them, the split solve parts covering every row once.
"""
import os
import subprocess

import numpy as np
import pytest

from helpers import make_problem
from plate_inverse_problem_amd import _native

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plate_inverse_problem_amd", "csrc")
EXE = os.path.join(CSRC, "..", "_lib", "asan", "symbolic_asan")


@pytest.fixture(scope="module")
def asan_exe():
    r = subprocess.run(["make", "-s", "-C", CSRC, "asan-host"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert os.path.exists(EXE)
    return EXE


def _active_pattern(p):
    active = [k for k in range(26) if not (p.material.is_mps and 6 <= k < 12)]
    keep = p.present[active].any(0) & (p.mats[active] != 0).any(0)     # as Problem._Engine
    idx = np.nonzero(keep)[0]
    rows, cols = p.rows[idx], p.cols[idx]
    colptr = np.zeros(p.mat_size + 1, np.int64)
    np.add.at(colptr, cols.astype(np.int64) + 1, 1)
    return np.cumsum(colptr).astype(np.int32), rows.astype(np.int32)


def _write(path, n, colptr, rowind, last):
    with open(path, "wb") as f:
        np.array([n], np.int32).tofile(f)
        np.array([rowind.size], np.int64).tofile(f)
        colptr.astype(np.int32).tofile(f)
        rowind.astype(np.int32).tofile(f)
        np.array([last.size], np.int32).tofile(f)
        last.astype(np.int32).tofile(f)


def _fnv(perm):
    h = 1469598103934665603
    for v in perm.tolist():
        h = ((h ^ (v & 0xFFFFFFFF)) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


# (leaf, ordering, symmetric, max_ns, md_delta, use_last)
OPTION_SETS = [
    (10000, 0, 1, 256, 4, 0),   # the engine above 512 frequencies (deep MMD tree)
    (200, 0, 1, 256, 4, 0),     # the engine up to 256 frequencies
    (1000, 0, 1, 256, 4, 0),    # the engine at 257-512 frequencies (C4's per-rank share)
    (2000, 0, 1, 256, 4, 0),    # the engine at 513-1,024 frequencies
    (96, 0, 1, 256, 4, 0),      # the width rule of round 3 at <= 512
    (16, 0, 1, 256, 4, 0),
    (10000, 0, 0, 256, 4, 0),   # general analysis (explicit-matrix solves)
    (96, 2, 1, 256, 0, 0),      # exact minimum degree leaves (rounds 1-3)
    (96, 0, 1, 8, 2, 1),        # support last, small supernodes
    (500, 1, 0, 0, 4, 0),       # natural order, no supernode split
]


@pytest.mark.parametrize("material,ny", [("isotropic", 3), ("sol", 4), ("orthotropic", 12), ("orthotropic", 25)])
def test_symbolic_under_asan_ubsan(asan_exe, tmp_path, material, ny):
    p = make_problem(material, ny=ny)
    colptr, rowind = _active_pattern(p)
    aU, aV, aW = p.averaging_vectors()
    sup = np.nonzero((aU != 0) | (aV != 0) | (aW != 0))[0].astype(np.int32)
    path = str(tmp_path / "pattern.bin")
    _write(path, p.mat_size, colptr, rowind, sup)
    sets = [s for s in OPTION_SETS if not (ny == 25 and s[1] == 1)]      # natural order at C3: too much fill
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([asan_exe, path] + [",".join(map(str, s)) for s in sets], capture_output=True, text=True,
                       env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 2 * len(sets), r.stdout[-2000:]
    for s, line, plan in zip(sets, lines[0::2], lines[1::2]):
        if int(line.split()[2]) > 1024:   # a front beyond the solve kernels' LDS staging: refused, as by libpfr
            assert plan.startswith("plan error") and "MAX_FRONT" in plan, (s, plan)
        else:
            assert plan == "plan ok 45", (s, plan)
        leaf, ordering, symmetric, max_ns, md_delta, use_last = s
        sym = _native.Symbolic(p.mat_size, colptr, rowind, leaf_size=leaf, ordering=ordering,
                               symmetric=bool(symmetric), max_ns=max_ns, md_delta=md_delta,
                               last=sup if use_last else None)
        st = sym.stats()
        v = line.split()
        assert v[0] != "error", line
        got = (int(v[0]), int(v[1]), int(v[2]), int(v[3]), int(v[4]), float(v[5]), int(v[6]), int(v[7]), int(v[8]))
        want = (st["n_fronts"], st["n_levels"], st["max_front"], st["total_rows"], st["nnz_lu"], st["factor_flops"],
                _fnv(sym.export("PERM")), st["n_dirichlet"], st["n_coupling"])
        assert got == want, (s, got, want)
