"""Diagnostic: per-wave timeline of the L21 row launches (k_offdiag_level) of one C3 sweep.

    PFR_LIB=plate_inverse_problem_amd/_lib/libpfr_wt.so PFR_LANES=1 python tools/wave_trace.py [--freqs 2048]
        [--out OUT.json]

(libpfr_wt.so: make -C plate_inverse_problem_amd/csrc OUT=../_lib/libpfr_wt.so OBJDIR=../_lib/obj_wt
EXTRA=-DPFR_WTRACE=1.)  Per launch (= level): waves with work, the launch's span, the waves' lifetimes
(median / 90th percentile / max), how late the last wave started, waves resident at once (mean over the span)
-- whether a level is bound by the length of each wave's work or by waiting for a slot -- and, for the slowest
10 % of its waves, the time in the source gathers, the left-looking prefix and the rest (each phase closed by a
wait for the wave's memory operations, which the production kernel overlaps).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--freqs", type=int, default=2048)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from helpers import make_problem
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    T = np.load(os.path.join(REPO, "tests", "golden", "c3_grad_truth.npz"))
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    sel = np.arange(args.freqs) * (4096 // args.freqs)
    eng = p.engine(args.freqs)
    eng.set_coefficients(_coeffs18(p._transform(), torch.as_tensor(T["theta"])).detach().numpy())
    dev = eng.device

    def sweep():
        w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        eng.sweep(torch.as_tensor(T["freqs"][sel], device=dev), _native.LOSS_MSE_LOG_AFC,
                  ref=torch.view_as_real(torch.as_tensor(T["ref"][sel].astype(np.complex128), device=dev)),
                  scale=1.0, loss=loss, w=torch.view_as_real(w))
        torch.cuda.synchronize()

    sweep()                                   # warm
    sv = eng.solvers[0]
    cap = 4 << 20
    sv.wave_trace_start(cap)
    sweep()
    rec = sv.wave_trace_fetch(cap).astype(np.int64)
    launch = rec[:, 3] >> 40
    tag = rec[:, 3] & ((1 << 40) - 1)
    rows = []
    for k in np.unique(launch):
        m = (launch == k) & (tag > 0) & (rec[:, 0] > 0)
        if not m.any():
            continue
        t0, t1 = rec[m, 0], rec[m, 1]
        life = (t1 - t0) * 10e-3                       # us (100 MHz)
        span = (t1.max() - t0.min()) * 10e-3
        late = (t0.max() - t0.min()) * 10e-3
        # phase clocks (sources / prefix; the rest = triangle + stores + setup), 10 ns units
        src = (rec[m, 2] >> 32) * 10e-3
        pre = (rec[m, 2] & 0xFFFFFFFF) * 10e-3
        slow = life >= np.percentile(life, 90)
        resident = life.sum() / span if span > 0 else 0.0
        rows.append(dict(launch=int(k), waves=int(m.sum()), span_us=float(span), life_med_us=float(np.median(life)),
                         life_p90_us=float(np.percentile(life, 90)), life_max_us=float(life.max()),
                         last_start_us=float(late), resident_mean=float(resident),
                         slow_src_us=float(src[slow].mean()), slow_pre_us=float(pre[slow].mean()),
                         slow_rest_us=float((life - src - pre)[slow].mean())))
    print(f"{'launch':>6} {'waves':>7} {'span':>8} {'life med':>9} {'p90':>8} {'max':>8} {'last start':>10} "
          f"{'resident':>9} | slowest 10 %: {'sources':>8} {'prefix':>8} {'rest':>8}")
    for r in rows:
        print(f"{r['launch']:6d} {r['waves']:7d} {r['span_us']:8.1f} {r['life_med_us']:9.1f} {r['life_p90_us']:8.1f} "
              f"{r['life_max_us']:8.1f} {r['last_start_us']:10.1f} {r['resident_mean']:9.1f} |               "
              f"{r['slow_src_us']:8.1f} {r['slow_pre_us']:8.1f} {r['slow_rest_us']:8.1f}")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
