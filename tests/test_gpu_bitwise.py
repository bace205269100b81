"""GPU: launch variants that must reproduce the default kernels BIT FOR BIT at C3 size.

C4's per-rank workload (512 frequencies of the C3 sweep, the block with the resonance) and a 2,048-frequency
chunk: with each variant the loss, the 18 gradient partials and fr must EQUAL the default path's -- the same
operations per entry in the same order, so a difference means a wrong index, a lost update or a race:
  * PFR_US2_TINY: the paired top-down pass one wave per front on the levels whose pivot blocks are <= 4 / 8
    (k_usolve2_tiny) against the workgroup kernel (k_usolve2_level);
  * PFR_OFF_PU_WAVES: the software-pipelined L21 prefix (k_offdiag_level<0, false, 3>) on every launch against
    none;
  * PFR_FRONT0: the bottom level fused into one kernel (k_front0: A11, L21 and the update block per frequency in
    registers) against the four class kernels (assembly, A11 LU, L21 rows, Schur update) on level 0;
  * PFR_FAC_GBIG / PFR_FAC_G_NS / PFR_FAC_G_WG: the A11 LU (k_factor_sym<G>) with 4 / 8 lane groups per wave on
    the levels with big pivot blocks, on the launches with few workgroups, and on every level, against 2
    everywhere;
  * PFR_RES_UNROLL: the residual walks with 8 entries per gather batch against 4.
The measured-slower variants of round 4 (dependency-driven passes, right-looking / shared-U11 L21 rows, prefix
batches, fused A11 gather, pipelined paired updates) were removed with their tests.
"""
import gc
import os

import numpy as np
import pytest
import torch

from helpers import make_problem, report

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _run(monkeypatch, lo, hi, fac_lds="-1", env=None):
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
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


def _same(tag, base, got):
    dl = abs(got[0] / base[0] - 1)
    dw = float(np.max(np.abs(got[1] - base[1])) / np.max(np.abs(base[1])))
    dfr = float(np.max(np.abs(got[2] / base[2] - 1)))
    report(tag, loss_rel=dl, w_rel=dw, fr_rel=dfr, flagged=got[4])
    assert got[4] == 0
    assert dl == 0 and dw == 0 and dfr == 0, (tag, dl, dw, dfr)


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_tiny_front_top_down_bitwise(monkeypatch, lo, hi):
    base = _run(monkeypatch, lo, hi, env={"PFR_US2_TINY": "0"})
    for tiny in ("4", "8"):
        _same(f"us2_tiny{tiny}_{lo}_{hi}", base, _run(monkeypatch, lo, hi, env={"PFR_US2_TINY": tiny}))


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_offdiag_pipelined_prefix_bitwise(monkeypatch, lo, hi):
    base = _run(monkeypatch, lo, hi, env={"PFR_OFF_PU_WAVES": "0"})
    _same(f"offdiag_pu3_{lo}_{hi}", base, _run(monkeypatch, lo, hi, env={"PFR_OFF_PU_WAVES": "1000000000"}))


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_front0_fused_bottom_level_bitwise(monkeypatch, lo, hi):
    base = _run(monkeypatch, lo, hi, env={"PFR_FRONT0": "0"})
    _same(f"front0_{lo}_{hi}", base, _run(monkeypatch, lo, hi, env={"PFR_FRONT0": "1"}))



@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_factor_lane_groups_bitwise(monkeypatch, lo, hi):
    base = _run(monkeypatch, lo, hi, fac_lds="0", env={"PFR_FAC_G_WG": "0", "PFR_FAC_GBIG": "2"})
    for gb, gns, wg in (("4", "64", "0"), ("8", "20", "0"), ("2", "64", "1024"), ("2", "64", "1000000000")):
        _same(f"fac_gbig{gb}_ns{gns}_wg{wg}_{lo}_{hi}", base, _run(
            monkeypatch, lo, hi, fac_lds="0", env={"PFR_FAC_G_WG": wg, "PFR_FAC_GBIG": gb, "PFR_FAC_G_NS": gns}))


@pytest.mark.parametrize("lo,hi", [(1024, 1536), (0, 2048)])
def test_residual_walk_unroll_bitwise(monkeypatch, lo, hi):
    base = _run(monkeypatch, lo, hi, env={"PFR_RES_UNROLL": "4"})
    _same(f"res_unroll8_{lo}_{hi}", base, _run(monkeypatch, lo, hi, env={"PFR_RES_UNROLL": "8"}))
