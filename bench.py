"""Benchmark: freq-solves/s (forward + adjoint) of the C3 workload on N GPUs.

BASELINE.json metric "freq-solves/sec (forward+adjoint) @20k DOF; achieved HBM
GB/s vs peak", config C3 (N = 1): orthotropic plate, ~20k DOF, 4096 frequencies,
forward + adjoint (loss + gradient), fp64; C4 (N > 1): the same 4096 frequencies
sharded across the N GPUs.

* one STEP = one loss + gradient evaluation (``getLossFunction`` +
  ``backward``) over the frequency sweep: per frequency assemble -> LU ->
  forward solves -> FR -> loss cotangent -> adjoint solves -> contraction;
* strong scaling (default, C4 as BASELINE.json defines it): ``--freqs`` (4096)
  frequencies in total, rank r sweeps its contiguous block
  ``shard_range(4096, r, N)`` (512 per rank at N = 8); one all-reduce (RCCL) of
  the loss/gradient partials per step.  ``--weak``: ``--freqs`` per rank.  With
  N > 1 a strong run also times the weak workload (4096 per rank) and reports it
  in the ``weak`` field;
* ``value`` = all frequencies of all ranks / (max-over-ranks seconds per step);
* each GPU runs ``lanes`` (default 2) solvers on their own HIP streams over
  contiguous halves of its frequencies, concurrently;
* ``roofline``: the dominant kernel class by device time -- at C3 with the MMD ordering
  ``k_offdiag_level`` (the L21 rows of the multifrontal factorisation, HBM-bound; within a few
  % of ``k_schur_sym_blk``): algorithmic bytes per launch (the solver's count: L21 stores +
  gathered children's entries + L11/U11 read, 16 B per complex entry) / average
  launch time, from HIP events that libpfr records around every launch on the
  lane's stream during one isolated lane-0 sweep of a full chunk right after the
  timed region (inside the timed region the lanes overlap, so a launch's duration
  there also contains the other lane's work: reported as ``concurrent_*``);
  ``traffic`` = measured HBM bytes per launch from the committed rocprofv3
  FETCH_SIZE/WRITE_SIZE passes (the newest profiles/rNN/pmc_traffic.json,
  gfx950-corrected); the whole factorisation (``factor_roofline``) and the
  triangular solves (``sptrsv_roofline``) beside it;
* ``cpu_baseline`` (rank 0, N = 1 only): the oracle (scipy SuperLU, one process
  per core) on a bounded sample of the same workload -- best-CPU (one
  factorisation per frequency, reused for the transpose solve) as ``value``, the
  reference-faithful count (a factorisation per primal / transpose bind, as the
  reference's JAX rules do) beside it;
* ``parity``: the oracle partials of the CPU leg against a GPU sweep of the same
  frequencies (full-size C3 parity, paid for by the CPU leg).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--freqs F] [--weak] [--ny NY]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

FP64_PEAK_TFLOPS = 78.6      # MI355X FP64 vector/matrix (spec; MI355X_MICROARCH.md lists no fp64 row)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec
# the newest round's committed PMC traffic summary (profiles/rNN/pmc_traffic.json)
PMC_FILE = (sorted(glob.glob(os.path.join(REPO, "profiles", "r[0-9][0-9]", "pmc_traffic.json")))
            or [os.path.join(REPO, "profiles", "r01", "pmc_traffic.json")])[-1]
# kernel classes of the factorisation (libpfr per-class HIP-event timings, pfr_last_kernel_timings
# order); the rocprof names of a class's kernels start with one of its prefixes
KERNELS = (("k_assemble_level", "k_front0"), ("k_factor_level", "k_factor_sym"), ("k_offdiag_level",), ("k_schur_sym_blk",),
           ("k_schur_level", "k_schur_sym_level"))
KERNEL_NAMES = ("k_assemble_level + k_front0 (level 0 fused)", "k_factor_level", "k_offdiag_level", "k_schur_sym_blk",
                "k_schur_sym_level / k_schur_level")
# every launch of the triangular solves: level passes, split update parts, the sliced bottom-up chain and
# the combination of its functional slices
SOLVE_KERNELS = ("k_lsolve", "k_usolve", "k_fn_combine")


def _pmc():
    try:
        return json.load(open(PMC_FILE))
    except (OSError, ValueError):
        return None


def pmc_traffic(chunk, symmetric):
    """Measured HBM bytes per launch of each factorisation kernel class, scaled to ``chunk``."""
    d = _pmc()
    if d is None or d.get("factorisation") != ("symmetric" if symmetric else "general"):
        return [None] * len(KERNELS)
    out = []
    for k in KERNELS:
        es = [e for name, e in d["kernels"].items() if name.startswith(k)]
        if not es:
            out.append(None)
            continue
        byts = sum(e["read_bytes"] + e["write_bytes"] for e in es)
        out.append(byts / sum(e["dispatches"] for e in es) * chunk / d["freqs_per_sweep"])
    return out


def pmc_solve_traffic(symmetric):
    """Measured HBM bytes per frequency of one sweep's triangular solves (every launch of the solve
    kernels; chunks counted by their k_chunk_start launches -- k_pad_freqs before round 6 --, one per chunk of
    freqs_per_sweep)."""
    d = _pmc()
    if d is None or d.get("factorisation") != ("symmetric" if symmetric else "general"):
        return None
    k = d["kernels"]
    sweeps = sum(e["dispatches"] for n, e in k.items() if n in ("k_chunk_start", "k_pad_freqs"))
    if not sweeps:
        return None
    byts = sum(e["read_bytes"] + e["write_bytes"] for n, e in k.items() if n.startswith(SOLVE_KERNELS))
    return byts / sweeps / d["freqs_per_sweep"]


def build_problem(ny, device, max_batch=None):
    from plate_inverse_problem_amd.Accelerometer import Accelerometer
    from plate_inverse_problem_amd.Geometry import Geometry, GeometryParams
    from plate_inverse_problem_amd.Material import get_material
    from plate_inverse_problem_amd.Problem import Problem
    acc = Accelerometer("AP1030")
    geom = Geometry("sh_i", acc, GeometryParams(100e-3, 20e-3, 2e-3, None, None), ny=ny)
    mat = get_material(1500.0, "orthotropic", E1=120e9, E2=8e9, G12=5e9, nu12=0.3, beta=0.01)
    return Problem(geom, mat, acc, device=device, max_batch=max_batch)


def cpu_baseline(prob, freqs, ref, theta, sample_per_core=128, faithful_per_core=24):
    """Oracle CPU sweeps on bounded samples (rank 0, N = 1): best-CPU and reference-faithful.
    Returns (baseline dict, (sample frequencies, loss_sum, w) of the best-CPU sample)."""
    from tests.helpers import oracle_for
    from oracle.plate_oracle import parallel_partials
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    cores = max(1, min(cores, os.cpu_count() or 1, 16))
    orc = oracle_for(prob)
    n = min(freqs.size, sample_per_core * cores)
    idx = np.linspace(0, freqs.size - 1, n).round().astype(int)
    t0 = time.perf_counter()
    loss_sum, w, _ = parallel_partials(orc, freqs[idx], ref[idx], "MSE_LOG_AFC", theta, n_workers=cores)
    dt = time.perf_counter() - t0
    # the reference's count: its JAX rules bind spsolve twice in the primal / linearisation and twice
    # transposed, each bind a fresh UMFPACK factorisation (Sparse.py:200-222, InnerState.h:276-288);
    # >= 3 survive XLA's CSE of the identical primal callbacks
    nf = min(freqs.size, faithful_per_core * cores)
    idf = np.linspace(0, freqs.size - 1, nf).round().astype(int)
    t0 = time.perf_counter()
    parallel_partials(orc, freqs[idf], ref[idf], "MSE_LOG_AFC", theta, n_workers=cores, factorisations=3)
    dtf = time.perf_counter() - t0
    out = {"value": n / dt, "unit": "freq-solves/s", "cores": cores, "kind": "port",
           "sample": f"{n} of the {freqs.size} frequencies (evenly spaced), forward+adjoint, one SuperLU "
                     f"factorisation per frequency reused for the transpose solve (best-CPU), every solve with "
                     f"UMFPACK's default refinement, {cores} processes, {dt:.1f} s",
           "reference_faithful": {"value": nf / dtf, "unit": "freq-solves/s", "cores": cores,
                                  "factorisations_per_frequency": 3,
                                  "sample": f"{nf} of the {freqs.size} frequencies, a fresh factorisation for the "
                                            f"primal solve and for each of the two transposed binds (the reference's "
                                            f"spsolve rules after CSE), {cores} processes, {dtf:.1f} s"}}
    return out, (freqs[idx], ref[idx], loss_sum, w)


def gpu_parity(prob, sample, theta):
    """The CPU leg's oracle partials (loss sum, 18 gradient partials w_k) against one GPU sweep of
    the same frequencies: full-size C3 parity."""
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    f, ref, loss_o, w_o = sample
    eng = prob.engine(f.size)
    c = _coeffs18(prob._transform(), torch.as_tensor(theta)).detach().numpy()
    eng.set_coefficients(c)
    dev = eng.device
    w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
    loss = torch.zeros(1, dtype=torch.float64, device=dev)
    eng.sweep(torch.as_tensor(f, device=dev), _native.LOSS_MSE_LOG_AFC,
              ref=torch.view_as_real(torch.as_tensor(ref.astype(np.complex128), device=dev)), scale=1.0 / f.size,
              loss=loss, w=torch.view_as_real(w))
    wg = eng.expand(w).cpu().numpy()
    lg = float(loss.item())
    return {"frequencies": int(f.size), "loss_rel": abs(lg - loss_o) / abs(loss_o),
            "grad_partials_rel": float(np.max(np.abs(wg - w_o)) / np.max(np.abs(w_o))),
            "measure": "oracle (SuperLU + UMFPACK-default refinement) loss sum and the 18 complex gradient "
                       "partials w_k = sum_f(-lam^T S_k x + e_k lam^T b0) against one GPU sweep of the same "
                       "frequencies; relative, max-norm over k"}


def strong_proxy(headline, ny, steps=10, warmup=2):
    """C4's per-rank work on this GPU, driver-timed: rank 0's block ``shard_range(4096, 0, 8)`` (512
    frequencies; every rank's block has the same work) as a loss + gradient sweep on a fresh engine sized for
    it, in a fresh process as a rank is (tools/strong_proxy.py --one).  share = its per-frequency rate over
    the headline's; predicted_c4 = 8 x the per-rank rate (the 304-B all-reduce per step left out)."""
    cmd = [sys.executable, os.path.join(REPO, "tools", "strong_proxy.py"), "--one", "512", "0", "--steps", str(steps),
           "--warmup", str(warmup), "--ny", str(ny)]
    t0 = time.perf_counter()
    res = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600)
    if res.returncode != 0:
        return {"error": f"tools/strong_proxy.py exited {res.returncode}"}
    r = json.loads(res.stdout.strip().splitlines()[-1])
    rate = r["freq_solves_per_s"]
    return {"freqs_per_rank": 512, "value": rate, "unit": "freq-solves/s", "ms_per_step": r["ms_per_step"],
            "steps": steps, "warmup": warmup, "share": rate / headline, "predicted_c4": 8 * rate,
            "lanes": r["lanes"], "chunk": r["chunk"], "wall_s": time.perf_counter() - t0,
            "measure": "rank 0's block of linspace(40, 600, 4096) for N = 8 (shard_range(4096, 0, 8)), loss + "
                       "gradient per step, a fresh process and engine; share = per-rank rate / the headline's"}


def timed(step, steps, warmup, world, device):
    """W untimed steps, then K steps bracketed by barrier + synchronize; max over ranks."""
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--freqs", type=int, default=4096, help="frequencies in total (strong) / per GPU (--weak)")
    ap.add_argument("--weak", action="store_true", help="--freqs per GPU instead of in total")
    ap.add_argument("--ny", type=int, default=25, help="mesh cells across the width (25 -> 19,353 DOF)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-strong-proxy", action="store_true", help="skip the 512-frequency per-rank sweep (C4 share)")
    ap.add_argument("--chunk", type=int, default=None, help="frequencies per chunk (default: from free HBM)")
    args = ap.parse_args()

    local = int(os.environ.get("LOCAL_RANK", 0))
    # rehearsal of the N > 1 path on one GPU (tests/test_gpu_bench_ranks.py): every rank on cuda:0,
    # gloo collectives; the driver's multi-GPU runs use the defaults (cuda:LOCAL_RANK, RCCL)
    if os.environ.get("PFR_BENCH_ONE_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    from plate_inverse_problem_amd.distributed import init_from_env, shard_range
    import plate_inverse_problem_amd.distributed as pdist
    rank, world, backend = init_from_env(device)       # under torch.distributed.run: always (RCCL)

    prob = build_problem(args.ny, device, args.chunk)
    theta_true = prob.parameters.copy()
    theta = theta_true * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1]))

    def workload(n_total):
        freqs = np.linspace(40.0, 600.0, n_total)
        lo, hi = shard_range(n_total, rank, world)
        ref = np.zeros(n_total, dtype=np.complex128)
        ref[lo:hi] = prob.solveForward(freqs[lo:hi], theta_true)          # synthetic measurement, phase 0
        loss_fn = prob.getLossFunction(freqs, ref, "MSE_LOG_AFC", distributed=backend is not None)

        def step():
            x = torch.tensor(theta, requires_grad=True)
            val = loss_fn(x)
            val.backward()
            return val.item(), x.grad
        return freqs, ref, lo, hi, step

    n_total = args.freqs * world if args.weak else args.freqs
    freqs, ref, lo, hi, step = workload(n_total)
    eng = prob.engine()
    solver = eng.solver
    # timed region: no device timing at all; per-phase HIP events in one extra untimed step, per-launch
    # events (which cost host time that delays the second lane's launches) in another
    eng.set_timing(False)
    n_coll0 = pdist.N_COLLECTIVES
    last = {}

    def step_acc():
        last["val"], last["grad"] = step()

    elapsed = timed(step_acc, args.steps, args.warmup, world, device)
    collectives = (pdist.N_COLLECTIVES - n_coll0) / (args.steps + args.warmup)
    eng.set_timing(True, kernels=False)
    step()
    torch.cuda.synchronize()
    phase = np.asarray(eng.last_timings(), dtype=np.float64)
    val = last["val"]
    # backward errors of the solves of this untimed step (same workload and theta as the timed steps;
    # checked on the device in every sweep)
    berr = eng.last_berr.cpu().numpy()
    check = {"measure": "componentwise backward error max_i |b - A x|_i / (|A||x| + |b|)_i per frequency "
                        "(UMFPACK's omega1), on the device in every sweep",
             "mode": eng.check_mode, "tol": eng.check_tol,
             "max_forward": float(np.nanmax(berr[:, 0])), "max_adjoint": float(np.nanmax(berr[:, 1])),
             "median_forward": float(np.nanmedian(berr[:, 0])),
             "flagged": int(np.count_nonzero(eng.last_flags)) if eng.last_flags is not None else None}
    eng.set_timing(True, kernels=True)
    step()
    torch.cuda.synchronize()
    kms, klaunch = eng.last_kernel_timings()
    ms_per_step = 1e3 * elapsed / args.steps
    value = n_total / (elapsed / args.steps)

    from plate_inverse_problem_amd import _native
    st = eng.stats
    nv = hi - lo

    # Kernel rooflines: one isolated sweep (lane 0 alone, its full chunk, same workload and
    # theta) right after the timed region, HIP events on lane 0's stream around every launch.
    # In the timed region the two lanes overlap, so per-launch durations there include the
    # other lane's kernels sharing the GPU (reported as "concurrent_*").
    chunk = solver.max_batch
    f_iso = torch.as_tensor(freqs[lo:lo + min(chunk, nv)], device=device)
    r_iso = torch.as_tensor(ref[lo:lo + f_iso.numel()], device=device)
    w_iso = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=device)
    l_iso = torch.zeros(1, dtype=torch.float64, device=device)
    with torch.cuda.stream(eng.streams[0]):
        solver.sweep(f_iso, _native.LOSS_MSE_LOG_AFC, ref=torch.view_as_real(r_iso), scale=1.0 / n_total, loss=l_iso,
                     w=torch.view_as_real(w_iso))
    torch.cuda.synchronize()
    iso_phase = solver.last_timings()
    iso_ms, iso_n = solver.last_kernel_timings()
    n_iso = f_iso.numel()
    alg_f = solver.alg_bytes().astype(float)             # algorithmic bytes per frequency, per kernel class
    alg_launch = alg_f * n_iso / np.maximum(iso_n, 1)
    ms_launch = iso_ms / np.maximum(iso_n, 1)
    gbs = alg_launch / (ms_launch * 1e-3) / 1e9
    kernels = KERNEL_NAMES
    traffic = pmc_traffic(chunk, eng.symmetric)
    dom = int(np.argmax(iso_ms))                         # the dominant kernel class
    fact_alg = float(alg_f.sum() * n_iso)
    fact_ms = float(iso_ms.sum())
    fact_tfs = st["factor_flops"] * n_iso / (iso_phase[0] * 1e-3) / 1e12
    fact_traffic = None if any(t is None and n > 0 for t, n in zip(traffic, iso_n)) else \
        float(sum(t * n for t, n in zip(traffic, iso_n) if n > 0))
    # triangular solves of the sweep: libpfr's count of the factor entries each pass must read (the
    # paired top-down pass reads U once for the adjoint and the rest of the forward solution), 16 B
    # each, plus rhs in / solution out; PMC traffic of the same kernels beside it
    sb = solver.solve_bytes().astype(float)
    trsv_bytes = n_iso * float(sb.sum())
    trsv_ms = iso_phase[1] + iso_phase[3]
    trsv_gbs = trsv_bytes / (trsv_ms * 1e-3) / 1e9
    trsv_traffic = pmc_solve_traffic(eng.symmetric)
    conc_launch = kms / np.maximum(klaunch, 1)
    out = {
        "metric": "freq-solves/sec (forward+adjoint) @20k DOF",
        "value": value,
        "unit": "freq-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (FE plate model built in-repo; reference FR = forward sweep at theta_true)",
        "config": {"workload": ("C3" if world == 1 else "C4") + ": orthotropic CFRP-like plate, sh_i strip "
                               f"100x20x2 mm + AP1030, {st['n']} DOF, {n_total} freqs in 40-600 Hz "
                               f"({'per GPU' if args.weak else 'in total'}, {nv} on rank 0), forward+adjoint, "
                               "loss MSE_LOG_AFC + gradient",
                   "n_dofs": st["n"], "freqs_total": n_total, "freqs_rank0": nv, "chunk": chunk,
                   "lanes": eng.n_lanes,
                   "factorisation": "symmetric: A = L U, U = diag(U) L^T implicit, Dirichlet nodes decoupled"
                                    if eng.symmetric else "general: A = L U",
                   "nnz_lu": st["nnz_lu"], "factor_gflop_per_freq": st["factor_flops"] / 1e9,
                   "parallelism": f"frequency shards x{world} + 1 all-reduce/step; {eng.n_lanes} concurrent "
                                  "solver lanes (HIP streams) per GPU",
                   "backend": backend, "collectives_per_step": collectives},
        "roofline": {"bound": "hbm", "kernel": kernels[dom], "achieved": gbs[dom], "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": gbs[dom] / HBM_PEAK_GBS, "traffic": traffic[dom],
                     "alg_bytes_per_launch": alg_launch[dom], "avg_launch_ms": ms_launch[dom],
                     "launches": int(iso_n[dom]), "measured": f"isolated lane-0 sweep of {n_iso} frequencies "
                     "(one chunk) after the timed region, HIP events per launch",
                     "concurrent_avg_launch_ms": conc_launch[dom]},
        "factor_roofline": {"bound": "hbm", "kernels": list(kernels), "ms": iso_ms.tolist(),
                            "alg_GBps": gbs.tolist(), "achieved": fact_alg / (fact_ms * 1e-3) / 1e9,
                            "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": fact_alg / (fact_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                            "alg_bytes": fact_alg, "traffic": fact_traffic, "frequencies": n_iso,
                            "fp64_TFLOPs": fact_tfs, "fp64_frac": fact_tfs / FP64_PEAK_TFLOPS,
                            "concurrent_ms_per_step": kms.tolist()},
        "sptrsv_roofline": {"bound": "hbm",
                            "kernel": "k_lsolve_level_z / k_lsolve_rows_z (one bottom-up chain: forward rhs + "
                                      "the functional's three vectors) + k_usolve2_level / k_usolve2_upd / "
                                      "k_usolve2_tiny (paired top-down) + k_fn_combine",
                            "achieved": trsv_gbs, "alg_bytes": trsv_bytes, "alg_bytes_per_freq": sb.tolist(),
                            "ms": trsv_ms, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": trsv_gbs / HBM_PEAK_GBS,
                            "traffic": None if trsv_traffic is None else trsv_traffic * n_iso,
                            "frequencies": n_iso},
        "phase_ms": {"factor": phase[0], "fwd_solves": phase[1], "functional": phase[2],
                     "adj_solves": phase[3], "contract": phase[4],
                     "note": "device ms per step summed over lanes; fwd_solves = the bottom-up chain over the "
                             "rhs reach and the loss support's reach (forward rhs + the functional's three vectors), "
                             "functional = its dot products + loss terms, adj_solves = the adjoint's bottom-up "
                             "combination + the paired top-down pass, contract = residual walks (checks and the "
                             "functional correction) + gradient contraction"},
        "loss": val,
        "backward_error": check,
    }
    if world > 1 and not args.weak:
        # the weak-scaling figure beside the strong one: 4096 frequencies per rank
        n_w = args.freqs * world
        _, _, lo_w, hi_w, step_w = workload(n_w)
        el_w = timed(step_w, args.steps, args.warmup, world, device)
        out["weak"] = {"value": n_w / (el_w / args.steps), "ms_per_step": 1e3 * el_w / args.steps,
                       "freqs_per_gpu": args.freqs, "freqs_total": n_w}
    if rank == 0 and world == 1 and not args.weak and args.freqs == 4096 and not args.no_strong_proxy:
        out["strong_proxy"] = strong_proxy(value, args.ny)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"], sample = cpu_baseline(prob, freqs, ref, theta)
        out["parity"] = gpu_parity(prob, sample, theta)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if backend is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
