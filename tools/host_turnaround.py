"""Host-side breakdown of the step-to-step turnaround of a loss + gradient loop (the GPU idles from the end of
step k's device work until step k+1's first launch).  Timestamps (perf_counter) at: the result copy returned
(end of loss_step k), bench-style step boundary, loss_step entry, each lane's pfr_sweep call entry.

    python tools/host_turnaround.py [n_freqs (512)] [steps (8)]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from plate_inverse_problem_amd import Problem as PM, _native  # noqa: E402

T = []
mark = lambda tag: T.append((tag, time.perf_counter()))  # noqa: E731

_orig_ls = PM._Engine.loss_step
_orig_sw = _native.Solver.sweep


def loss_step(self, *a, **k):
    mark("loss_step_in")
    r = _orig_ls(self, *a, **k)
    mark("loss_step_out")
    return r


def sweep(self, *a, **k):
    mark("native_sweep_in")
    r = _orig_sw(self, *a, **k)
    mark("native_sweep_out")       # the sweep's launches enqueued (host side)
    return r


PM._Engine.loss_step = loss_step
_native.Solver.sweep = sweep

# finer marks (HT_FINE=1): engine lookup, coefficient set, the lane runner, the per-lane set_check, stream waits
if os.environ.get("HT_FINE") == "1":
    import threading

    def _wrap(owner, name, tag):
        orig = getattr(owner, name)

        def f(*a, **k):
            main = threading.current_thread() is threading.main_thread()
            mark(tag + ("" if main else "@pool"))
            return orig(*a, **k)
        setattr(owner, name, f)
    _wrap(PM._Engine, "set_coefficients", "set_coef_in")
    _wrap(PM._Engine, "_run", "run_in")
    _wrap(_native.Solver, "set_check", "set_check_in")
    _wrap(torch.cuda.Stream, "wait_stream", "wait_stream_in")
    _wrap(PM.Problem, "engine", "engine_in")
    PM._HT = mark


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    p = bench.build_problem(25, torch.device("cuda", 0))
    th = p.parameters.copy()
    freqs = np.linspace(40.0, 600.0, 4096)[:n]
    ref = p.solveForward(freqs, th)
    fn = p.getLossFunction(freqs, ref, "MSE_LOG_AFC")
    theta = th * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1]))

    def step():
        mark("step_in")
        x = torch.tensor(theta, requires_grad=True)
        v = fn(x)
        mark("forward_done")
        v.backward()
        mark("backward_done")
        return v.item(), x.grad

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    T.clear()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    # per step: time from the previous loss_step_out (result on the host) to this step's first native sweep call
    outs = [t for tag, t in T if tag == "loss_step_out"]
    rows = []
    for i in range(1, steps):
        t_prev = outs[i - 1]
        seg = [(tag, t) for tag, t in T if t > t_prev][:24]
        first_native = next(t for tag, t in seg if tag == "native_sweep_in")
        row = {}
        for tag, t in seg:
            row.setdefault(tag, round((t - t_prev) * 1e6, 1))     # first occurrence of each tag
        rows.append(row)
        rows[-1]["first_native_us"] = round((first_native - t_prev) * 1e6, 1)
    for r in rows:
        print(r)
    if os.environ.get("HT_DUMP"):
        # absolute CLOCK_MONOTONIC ns of every mark (perf_counter on Linux), to line up with a rocprofv3 kernel trace
        import json
        off = time.monotonic_ns() - time.perf_counter_ns()
        json.dump([(tag, int(t * 1e9) + off) for tag, t in T], open(os.environ["HT_DUMP"], "w"))
    print("mean host time from result to the next step's first native sweep call: %.1f us"
          % np.mean([r["first_native_us"] for r in rows]))
    ins = [t for tag, t in T if tag == "native_sweep_in"]
    outs_n = [t for tag, t in T if tag == "native_sweep_out"]
    print("mean host enqueue time of one lane's sweep (pfr_sweep call to return): %.1f us"
          % (1e6 * np.mean(np.subtract(outs_n, ins))))


if __name__ == "__main__":
    main()
