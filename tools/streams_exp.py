"""Experiment: S solvers (chunk C each) sweeping 4096 frequencies on S HIP streams concurrently.

Measures loss+gradient sweep time of the C3 workload for a few (S, C) configurations.
Usage (GPU box): python tools/streams_exp.py
"""
import sys
import time

sys.path.insert(0, '/root/repo')
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bench import build_problem  # noqa: E402
from plate_inverse_problem_amd import _native  # noqa: E402
from plate_inverse_problem_amd.Problem import _coeffs18  # noqa: E402

dev = torch.device('cuda', 0)
freqs = np.linspace(40, 600, 4096)
f_all = torch.as_tensor(freqs, device=dev)
p0 = build_problem(25, dev)
ref = torch.as_tensor(p0.solveForward(freqs).astype(np.complex128), device=dev)
th = p0.parameters * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1]))
c = _coeffs18(p0._transform(), torch.as_tensor(th)).numpy()
p0._engine = None
torch.cuda.empty_cache()


def run(engines, streams):
    cur = torch.cuda.current_stream(dev)
    n = len(engines)
    per = 4096 // n
    outs = []
    for i, (e, s) in enumerate(zip(engines, streams)):
        s.wait_stream(cur)
        sl = slice(i * per, (i + 1) * per)
        with torch.cuda.stream(s):
            w = torch.zeros(18, dtype=torch.complex128, device=dev)
            loss = torch.zeros(1, dtype=torch.float64, device=dev)
            e.solver.sweep(f_all[sl].contiguous(), _native.LOSS_IDS['MSE_LOG_AFC'],
                           ref=torch.view_as_real(ref[sl].contiguous()), scale=1 / 4096, loss=loss,
                           w=torch.view_as_real(w))
            outs.append((loss, w))
    for s in streams:
        cur.wait_stream(s)
    return sum(o[0] for o in outs), sum(o[1] for o in outs)


results = {}
for n_s, chunk in [(1, 2048), (2, 1024), (4, 512), (2, 2048)]:
    probs = [build_problem(25, dev) for _ in range(n_s)]
    engines = []
    for p in probs:
        p._max_batch = chunk
        e = p.engine(4096 // n_s)
        e.set_coefficients(c)
        engines.append(e)
    streams = [torch.cuda.Stream(dev) for _ in range(n_s)]
    for _ in range(2):
        run(engines, streams)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(3):
        lv, wv = run(engines, streams)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / 3
    results[(n_s, chunk)] = (dt, lv.item(), wv.cpu())
    print(f"{n_s} solvers x chunk {chunk}: {dt * 1e3:.1f} ms per 4096  ({4096 / dt:.0f} freq-solves/s)  "
          f"loss {lv.item():.12e}", flush=True)
    del engines, probs, streams
    torch.cuda.empty_cache()
base = results[(1, 2048)]
for k, (dt, lv, wv) in results.items():
    print(k, "loss rel diff", abs(lv - base[1]) / abs(base[1]), "w rel diff",
          float((wv - base[2]).abs().max() / base[2].abs().max()))
