"""GPU: the dependency-driven passes over the narrow top of the elimination tree (PFR_FLOW bits: 1 the paired
top-down solve, 2 the sliced bottom-up chain, 4 the factorisation) at C3 size against the level-by-level
launches and the extended-precision truth.

C4's per-rank workload (512 frequencies of the C3 sweep, the block with the resonance) and a 2,048-frequency
chunk, with the global-memory A11 LU on every level (PFR_FAC_LDS=0: the flow's A11 tasks use it, and the LDS
LU of the level launches rounds differently): with every flow the loss, the 18 gradient partials and fr must
EQUAL the level-launch results -- the same operations per entry in the same order (the A11 LU's row-to-wave
map and, for the small update blocks, the Schur kernel differ, not the arithmetic), so any hand-off that let a
task read a stale or unfinished value shows as a difference.  With the default LDS LU on the level launches,
fr at the fixture frequencies inside the block must lie within the accuracy class of the reference's refined
solves against the truth (2e-7: the oracle's refined SuperLU is within 1.65e-7 over the 4,096 frequencies,
c3_grad_truth.npz; the corrected static-pivot fr moves by ~1e-7 with the rounding of the pivot-block LU).
"""
import gc
import os

import numpy as np
import pytest
import torch

from helpers import make_problem, report

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _run(monkeypatch, flow, lo, hi, fac_lds="0", env=None):
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    monkeypatch.setenv("PFR_FLOW", str(flow))
    monkeypatch.setenv("PFR_FAC_LDS", fac_lds)
    for k, v in (env or {}).items():
        monkeypatch.setenv(k, v)
    T = np.load(os.path.join(GOLDEN, "c3_grad_truth.npz"))
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    try:
        sel = np.arange(lo, hi)
        f, ref = T["freqs"][sel], T["ref"][sel]
        eng = p.engine(sel.size)
        c = _coeffs18(p._transform(), torch.as_tensor(T["theta"])).detach().numpy()
        eng.set_coefficients(c)
        dev = eng.device
        w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        flags = torch.zeros(sel.size, dtype=torch.int32, device=dev)
        eng.sweep(torch.as_tensor(f, device=dev), _native.LOSS_MSE_LOG_AFC,
                  ref=torch.view_as_real(torch.as_tensor(ref.astype(np.complex128), device=dev)), scale=1.0 / sel.size,
                  loss=loss, w=torch.view_as_real(w), flags=flags)
        F = np.load(os.path.join(GOLDEN, "c3_truth.npz"))
        inside = (F["index"] >= lo) & (F["index"] < hi)
        fr = p.solveForward(F["freqs"][inside])
        out = (float(loss.item()), eng.expand(w).cpu().numpy(), fr, F["fr_true"][inside], int(flags.count_nonzero()))
        return out
    finally:
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_flows_match_level_launches(monkeypatch, lo, hi):
    base = _run(monkeypatch, 0, lo, hi)
    for flow in (1, 2, 4, 7):
        got = _run(monkeypatch, flow, lo, hi)
        dl = abs(got[0] / base[0] - 1)
        dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
        dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
        err = float(np.max(np.abs(got[2] / got[3] - 1)))
        report(f"flow{flow}_{lo}_{hi}", loss_rel=dl, w_rel=dw, fr_rel=dfr, fr_vs_truth=err, flagged=got[4])
        assert got[4] == 0, (flow, got[4])
        assert dl == 0 and dw == 0 and dfr == 0, (flow, dl, dw, dfr)
        assert err < 2e-7, (flow, err)


def test_factor_flow_default_lds_accuracy(monkeypatch):
    """The factorisation flow against the default level launches (LDS A11 LU on their few-workgroup levels):
    both within the refined solves' accuracy class of the truth, loss and partials to that class too."""
    base = _run(monkeypatch, 0, 1024, 1536, fac_lds="-1")
    got = _run(monkeypatch, 7, 1024, 1536, fac_lds="-1")
    e0 = float(np.max(np.abs(base[2] / base[3] - 1)))
    e1 = float(np.max(np.abs(got[2] / got[3] - 1)))
    dl = abs(got[0] / base[0] - 1)
    dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
    report("flow7_default_lds", fr_vs_truth_level=e0, fr_vs_truth_flow=e1, loss_rel=dl, w_rel=dw)
    assert got[4] == 0 and e0 < 2e-7 and e1 < 2e-7
    assert dl < 1e-7 and dw < 4e-7


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_offdiag_right_looking_bitwise(monkeypatch, lo, hi):
    """k_offdiag_rl (PFR_OFF_RL: the L21 rows right-looking, the row in registers) performs k_offdiag_level's
    operations per entry in the same order: loss, partials and fr identical, on the narrow (512) and the
    bench's (2,048) engine."""
    base = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_OFF_RL": "0"})
    for rl in ("16", "32", "116", "124"):       # one row per wave; 100 + n: an item's two rows per wave
        got = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_OFF_RL": rl})
        dl = abs(got[0] / base[0] - 1)
        dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
        dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
        report(f"offdiag_rl{rl}_{lo}_{hi}", loss_rel=dl, w_rel=dw, fr_rel=dfr, flagged=got[4])
        assert got[4] == 0
        assert dl == 0 and dw == 0 and dfr == 0, (rl, dl, dw, dfr)


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_tiny_front_top_down_bitwise(monkeypatch, lo, hi):
    """k_usolve2_tiny (PFR_US2_TINY: the paired top-down pass one wave per front on the levels whose pivot blocks
    are at most 4 / 8) performs k_usolve2_level's operations in the same order: identical results."""
    base = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_US2_TINY": "0"})
    for tiny in ("4", "8", "16", "32"):   # > 8: k_usolve2_wave
        got = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_US2_TINY": tiny})
        dl = abs(got[0] / base[0] - 1)
        dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
        dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
        report(f"us2_tiny{tiny}_{lo}_{hi}", loss_rel=dl, w_rel=dw, fr_rel=dfr, flagged=got[4])
        assert got[4] == 0
        assert dl == 0 and dw == 0 and dfr == 0, (tiny, dl, dw, dfr)


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_offdiag_shared_u11_bitwise(monkeypatch, lo, hi):
    """k_offdiag_shu (PFR_OFF_SHU: L21 rows with U11 staged once per workgroup in LDS, on the levels with fewer
    (item, group) waves than the knob) performs k_offdiag_level's operations in the same order: identical."""
    base = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_OFF_SHU": "0"})
    for shu in ("4096", "1000000000"):
        got = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_OFF_SHU": shu})
        dl = abs(got[0] / base[0] - 1)
        dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
        dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
        report(f"offdiag_shu{shu}_{lo}_{hi}", loss_rel=dl, w_rel=dw, fr_rel=dfr, flagged=got[4])
        assert got[4] == 0
        assert dl == 0 and dw == 0 and dfr == 0, (shu, dl, dw, dfr)


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_offdiag_prefix_batches_bitwise(monkeypatch, lo, hi):
    """PFR_OFF_PU: the L21 prefix loop in batches of 4 / 8 pivots whose loads are issued first (on the launches
    with fewer waves than PFR_OFF_PU_WAVES) -- the same products in the same order: identical results."""
    base = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_OFF_PU_WAVES": "0"})
    for pu in ("3", "4", "8"):   # 3: software-pipelined
        got = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_OFF_PU": pu, "PFR_OFF_PU_WAVES": "1000000000"})
        dl = abs(got[0] / base[0] - 1)
        dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
        dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
        report(f"offdiag_pu{pu}_{lo}_{hi}", loss_rel=dl, w_rel=dw, fr_rel=dfr, flagged=got[4])
        assert got[4] == 0
        assert dl == 0 and dw == 0 and dfr == 0, (pu, dl, dw, dfr)


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_paired_update_pipelined_bitwise(monkeypatch, lo, hi):
    """PFR_US2_PP: the paired top-down pass's split update parts software-pipelined (the next chunk's loads before
    the current chunk's products): identical results."""
    base = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_US2_PP": "0"})
    got = _run(monkeypatch, 0, lo, hi, fac_lds="-1", env={"PFR_US2_PP": "1"})
    dl = abs(got[0] / base[0] - 1)
    dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
    dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
    report(f"us2_pp_{lo}_{hi}", loss_rel=dl, w_rel=dw, fr_rel=dfr, flagged=got[4])
    assert got[4] == 0
    assert dl == 0 and dw == 0 and dfr == 0, (dl, dw, dfr)
