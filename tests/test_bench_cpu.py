"""CPU: bench.py's host-side pieces (no GPU): the committed PMC traffic summary it reads for the
roofline's `traffic` fields, and the reference-faithful CPU count's oracle option."""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def test_pmc_traffic_from_committed_profile():
    import bench
    d = json.load(open(bench.PMC_FILE))
    assert d["factorisation"] == "symmetric" and d["freqs_per_sweep"] == 2048
    t = bench.pmc_traffic(2048, True)
    # every class the profiled run launched
    assert len(t) == len(bench.KERNELS) and all(v is not None and v > 0 for v in t)
    # per-launch traffic of the Schur block class within 1.0x .. 1.5x its algorithmic bytes with the
    # round-3 MMD ordering (0.96 GB per launch at 2,048 frequencies: 33.6 GB over 35 level launches)
    assert 0.96e9 < t[3] < 1.5 * 0.96e9
    s = bench.pmc_solve_traffic(True)
    # solves: more than the 13.4 MB per frequency they must read (MMD ordering), less than 3x that
    assert 13.4e6 < s < 3 * 13.4e6
    assert bench.pmc_traffic(2048, False) == [None] * len(bench.KERNELS)   # no general-mode profile


def test_newest_round_profile_is_used():
    import bench
    rounds = sorted(p for p in os.listdir(os.path.join(REPO, "profiles")) if p.startswith("r"))
    assert os.path.dirname(bench.PMC_FILE).endswith(rounds[-1])


def test_reference_faithful_count_has_the_same_partials():
    from helpers import make_problem, oracle_for
    from oracle.plate_oracle import frequency_partials
    p = make_problem("isotropic", ny=2)
    o = oracle_for(p)
    f = np.array([120.0, 333.0])
    ref = o.fr(f, p.parameters) * 1.01
    a = frequency_partials(o, f, ref, "MSE_LOG_AFC", p.parameters)
    b = frequency_partials(o, f, ref, "MSE_LOG_AFC", p.parameters, factorisations=3)
    assert np.isclose(a[0], b[0], rtol=1e-13) and np.allclose(a[1], b[1], rtol=1e-10, atol=1e-14)
