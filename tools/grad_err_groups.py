"""Where the GPU gradient error comes from: the C3 loss + gradient partials per 64-frequency group of the
bench's 4,096-frequency sweep against the extended-precision truth (tests/golden/c3_grad_truth.npz).

    python tools/grad_err_groups.py [--out OUT.json] [--check MODE]

Per group g (64 consecutive frequencies): the unscaled partial sums sum_{f in g} w_f of one GPU sweep
over the group against the truth's; printed as each group's error in units of max_k |sum_all w*_k|
(the normaliser of the test's relative error), largest first, plus the whole-sweep error.
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
    ap.add_argument("--out", default=None)
    ap.add_argument("--check", type=int, default=None, help="PFR_CHECK_* mode for the sweeps (default: engine's)")
    ap.add_argument("--group", type=int, default=64)
    args = ap.parse_args()
    from helpers import make_problem
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    T = np.load(os.path.join(REPO, "tests", "golden", "c3_grad_truth.npz"))
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    theta = np.asarray(T["theta"])
    eng = p.engine(4096)
    if args.check is not None:
        eng.set_check(args.check)
    c = _coeffs18(p._transform(), torch.as_tensor(theta)).detach().numpy()
    eng.set_coefficients(c)
    dev = eng.device

    def sweep(sel):
        f = torch.as_tensor(T["freqs"][sel], device=dev)
        ref = torch.as_tensor(T["ref"][sel].astype(np.complex128), device=dev)
        w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        eng.sweep(f, _native.LOSS_MSE_LOG_AFC, ref=torch.view_as_real(ref), scale=1.0, loss=loss,
                  w=torch.view_as_real(w))
        return float(loss.item()), eng.expand(w).cpu().numpy()

    wt_all = T["w_true"].sum(0)
    norm = np.max(np.abs(wt_all))
    l_all, w_all = sweep(np.arange(4096))
    rows = []
    G = args.group
    for g in range(4096 // G):
        sel = np.arange(g * G, (g + 1) * G)
        l, w = sweep(sel)
        wt = T["w_true"][sel].sum(0)
        wo = T["w_oracle"][sel].sum(0)
        rows.append({"group": g, "f0": float(T["freqs"][sel[0]]), "err": float(np.max(np.abs(w - wt)) / norm),
                     "err_oracle": float(np.max(np.abs(wo - wt)) / norm),
                     "w_share": float(np.max(np.abs(wt)) / norm),
                     "fr_max": float(T["fr_true"][sel].max()),
                     "err_vec": (w - wt)[[12, 13, 14, 16, 17]].tolist() if False else None})
    rows.sort(key=lambda r: -r["err"])
    out = {"check_mode": eng.check_mode, "whole_sweep_err": float(np.max(np.abs(w_all - wt_all)) / norm),
           "whole_sweep_err_oracle": float(np.max(np.abs(T["w_oracle"].sum(0) - wt_all)) / norm),
           "sum_group_errs": float(sum(r["err"] for r in rows)), "groups": rows}
    print(f"whole sweep: gpu {out['whole_sweep_err']:.2e}  oracle {out['whole_sweep_err_oracle']:.2e}")
    for r in rows[:12]:
        print(f"group {r['group']:3d} {r['f0']:7.2f} Hz  err {r['err']:.2e}  oracle {r['err_oracle']:.2e}  "
              f"|w| share {r['w_share']:.2e}  fr max {r['fr_max']:.2f}")
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
