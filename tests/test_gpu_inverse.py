"""GPU: solveInverse end to end (reference cpu_benchmark.py flow, small mesh)."""
import numpy as np
import pytest

from helpers import make_problem

pytestmark = pytest.mark.gpu


def test_gd_inverse_runs_and_logs(tmp_path):
    """cpu_benchmark.py:63-66: relative start [0.1, 0.1, 0.2], MSE_LOG_AFC, gd, compression 200."""
    p = make_problem("isotropic", ny=4, device="cuda:0")
    freq = np.linspace(40, 600, 600)
    fr = p.solveForward(freq)
    res = p.solveInverse([0.1, 0.1, 0.2], 'MSE_LOG_AFC', 'gd', ref_fr=[freq, fr], use_rel=True,
                         compression=(True, 200), log=True, report=True, uid='t', log_dir=str(tmp_path),
                         N_steps=5, h=0.001, f_min=1e-10)
    assert len(res.f_history) == 5 and np.all(np.isfinite(res.x))
    assert (tmp_path / 't.txt').exists() and (tmp_path / 't.npz').exists()
    log = np.load(tmp_path / 't.npz')
    assert log['x'].shape == (6, 3) and log['f'].shape == (6,)


def test_lbfgs_recovers_parameters():
    """C5-style: scaled L-BFGS from a perturbed start (inside the basin: the FR
    misfit is multimodal once resonances move past each other) recovers theta_true."""
    p = make_problem("orthotropic", ny=4, device="cuda:0")
    freq = np.linspace(40, 600, 256)
    fr = p.solveForward(freq)
    res = p.solveInverse([0.03, -0.03, 0.04, 0.02, 0.1], 'MSE_LOG_AFC', 'lbfgs', ref_fr=[freq, fr],
                         use_rel=True, use_scaling=True, log=False, report=False, N_steps=40)
    rel = np.abs(res.x - p.parameters) / p.parameters
    assert res.f < 1e-5 * res.f_history[0]
    assert rel[0] < 1e-3 and rel[2] < 1e-3                # E1, G12: the well-identified moduli of the strip
