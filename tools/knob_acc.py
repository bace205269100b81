"""C3 fr against the extended-precision fixture (tests/golden/c3_truth.npz) for several launch-knob settings:
the corrected fr of the bench's 4,096-frequency sweep and the raw / corrected fr of the 32 fixture frequencies
with their backward errors.

    python tools/knob_acc.py KNOB=V[,KNOB=V] ...
"""
import gc
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def main():
    import torch
    from helpers import make_problem
    T = np.load(os.path.join(REPO, "tests", "golden", "c3_truth.npz"))
    freqs = np.linspace(40.0, 600.0, 4096)
    idx = T["index"]
    for cfg in sys.argv[1:] or [""]:
        env = dict(kv.split("=") for kv in cfg.split(",") if kv)
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        p = make_problem("orthotropic", ny=25, device="cuda:0")
        fr = p.solveForward(freqs)
        e = np.abs(fr[idx] / T["fr_true"] - 1)
        fr_raw, berr, flags = p.solveForwardChecked(T["freqs"], correct=False)
        er = np.abs(fr_raw / T["fr_true"] - 1)
        print("%-24s sweep: max %.2e median %.2e (%.1f Hz) | raw: max %.2e median %.2e | berr max %.1e flags %d"
              % (cfg or "default", e.max(), np.median(e), T["freqs"][e.argmax()], er.max(), np.median(er),
                 berr.max(), int(np.count_nonzero(flags))), flush=True)
        print("   per freq (sweep):", " ".join("%.1e" % x for x in e))
        print("   per freq (raw):  ", " ".join("%.1e" % x for x in er))
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


if __name__ == "__main__":
    main()
