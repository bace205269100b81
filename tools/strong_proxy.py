"""One-GPU proxy of C4's strong scaling (BASELINE.json configs[3]: C3's 4,096 frequencies sharded
across 8 GPUs, 512 per rank): loss + gradient throughput of C3 sweeps of 512, 1,024, 2,048 and
4,096 frequencies -- the per-rank work at N = 8, 4, 2, 1 -- each the contiguous block rank 0 would
own (``shard_range(4096, 0, N)``), on a fresh engine sized for it (as a rank's engine is).

    python tools/strong_proxy.py [--out profiles/r03/strong_proxy.json] [--steps 8]

Prints one line per size and writes the JSON: freq-solves/s, ms per step, the ratio of the
per-frequency rate to the 4,096 one (the parallel efficiency a SCALE run can at most reach when
the all-reduce is free) and the predicted N-GPU strong-scaling value (N x the per-rank rate).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def measure(n_rank, steps, warmup, ny, lanes=None, spread=False):
    import bench
    from plate_inverse_problem_amd.distributed import shard_range
    if lanes is not None:
        os.environ["PFR_LANES"] = str(lanes)
    prob = bench.build_problem(ny, torch.device("cuda", 0))
    theta_true = prob.parameters.copy()
    theta = theta_true * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1]))
    world = 4096 // n_rank
    freqs_all = np.linspace(40.0, 600.0, 4096)
    lo, hi = shard_range(4096, 0, world)
    freqs = np.linspace(40.0, 600.0, n_rank) if spread else freqs_all[lo:hi]
    ref = prob.solveForward(freqs, theta_true)
    loss_fn = prob.getLossFunction(freqs, ref, "MSE_LOG_AFC")

    def step():
        x = torch.tensor(theta, requires_grad=True)
        loss_fn(x).backward()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    eng = prob.engine()
    out = {"freqs_per_rank": n_rank, "ms_per_step": 1e3 * dt, "freq_solves_per_s": n_rank / dt,
           "lanes": eng.n_lanes, "chunk": eng.max_batch}
    del prob, eng, loss_fn
    gc.collect()
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--ny", type=int, default=25)
    ap.add_argument("--sizes", default="4096,2048,1024,512")
    ap.add_argument("--lanes", default="", help="comma list of lane counts to try per size (default: engine's)")
    ap.add_argument("--spread", action="store_true", help="n frequencies over the whole band instead of rank 0's block")
    ap.add_argument("--one", type=int, nargs=2, default=None, metavar=("N", "LANES"),
                    help="measure one size in this process (LANES 0: the engine's choice) and print its JSON")
    a = ap.parse_args()
    if a.one is not None:
        torch.cuda.set_device(0)
        print(json.dumps(measure(a.one[0], a.steps, a.warmup, a.ny, a.one[1] or None, a.spread)), flush=True)
        return
    # every size in a fresh process, as every rank is (an engine built after a larger one was freed in the
    # same process measured up to 12 % slower)
    rows = []
    lanes_list = [int(v) for v in a.lanes.split(",") if v] or [0]
    for n in [int(v) for v in a.sizes.split(",")]:
        for ln in lanes_list:
            cmd = [sys.executable, os.path.abspath(__file__), "--one", str(n), str(ln), "--steps", str(a.steps),
                   "--warmup", str(a.warmup), "--ny", str(a.ny)] + (["--spread"] if a.spread else [])
            res = subprocess.run(cmd, stdout=subprocess.PIPE, text=True, timeout=600)
            if res.returncode != 0:
                sys.exit(res.returncode)
            r = json.loads(res.stdout.strip().splitlines()[-1])
            rows.append(r)
            print(json.dumps(r), flush=True)
    base = {}
    for r in rows:
        if r["freqs_per_rank"] == 4096:
            base[r["lanes"]] = r["freq_solves_per_s"]
    ref_rate = max(base.values()) if base else None
    best = {}
    for r in rows:
        n = r["freqs_per_rank"]
        if n not in best or r["freq_solves_per_s"] > best[n]["freq_solves_per_s"]:
            best[n] = r
    summary = []
    for n, r in sorted(best.items()):
        world = 4096 // n
        eff = r["freq_solves_per_s"] / ref_rate if ref_rate else None
        summary.append({"freqs_per_rank": n, "n_gpus": world, "per_rank_rate": r["freq_solves_per_s"],
                        "rate_vs_4096": eff, "predicted_strong_value": world * r["freq_solves_per_s"],
                        "lanes": r["lanes"], "chunk": r["chunk"]})
    out = {"workload": "C3 loss + gradient (MSE_LOG_AFC), orthotropic, ny=25, rank 0's block of "
                       "linspace(40, 600, 4096) for N = 4096 / freqs_per_rank",
           "runs": rows, "summary": summary,
           "note": "per-rank throughput on one MI355X; predicted_strong_value = N x per-rank rate (all-reduce of "
                   "304 B per step not included)"}
    print(json.dumps({"summary": summary}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
