"""Full-size gradient parity: the C3 loss + gradient against extended-precision truth, and C4's per-rank
workload at C3 size.

Fixture: ``tests/golden/c3_grad_truth.npz`` (``tests/golden/make_c3_grad_truth.py``) -- per frequency of
the bench's 4,096-frequency C3 sweep the extended-precision loss term and the 18 complex gradient
partials ``w_f,k = -lam^T S_k x + e_k lam^T b0`` (``A^T lam = l'(fr) d fr / d x``, the non-conjugate
transpose of ``Sparse.py:211-219`` / ``InnerState.h:183-185``), and the same from the fp64 oracle
(SuperLU + UMFPACK's default refinement, the reference's solver configuration).  The measurement ``ref``
is the extended-precision fr at theta_true.

Measure: relative max-norm error of the partials, ``max_k |w_k - w*_k| / max_k |w*_k|`` with
``w = sum_S w_f / |S|`` over a frequency set S, and the relative error of the loss and of the theta
gradient.  Bound: the GPU partials, the theta gradient and the loss within W_RTOL / LOSS_RTOL (3e-8) of the
truth, absolute (no allowance from the oracle's own error; VERDICT round 3 asked for 2e-7).

C4 (BASELINE.json configs[3]): a rank of the 8-GPU run sweeps the 512-frequency block
``shard_range(4096, r, 8)``; a fresh engine sized for it takes the narrow-sweep path (2 lanes of 256, the
leaf-1,000 ordering, the A11 LU in LDS on its few-workgroup levels).  Block 2
holds the resonance (sample 1179).
"""
import gc
import os

import numpy as np
import pytest
import torch

from helpers import make_problem, report

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
# gradient partials against the extended-precision truth.  VERDICT round 3 asked for 2e-7; round 4 (the solve-error
# scale of the cotangent) measured 1.2-2.5e-8 and bounded at 6e-8.  Round 5 (compensated correction residual)
# measures partials 6.5e-9 .. 8.4e-9, theta gradient 4.3e-9 .. 1.6e-8, loss 5.9e-9 .. 7.3e-9 on every set
# (gpurun_out/r5i_tests; the fp64 oracle: 0.9-2.7e-8), so both bounds are 3e-8, with no oracle allowance
W_RTOL = 3e-8
LOSS_RTOL = 3e-8
FR_RTOL_C3 = 1e-7          # fr against c3_truth.npz (functional correction on, as in test_gpu_fullsize)


def _truth():
    return np.load(os.path.join(GOLDEN, "c3_grad_truth.npz"))


def _wrel(w, wt):
    return float(np.max(np.abs(w - wt)) / np.max(np.abs(wt)))


def _gpu_partials(p, freqs, ref, theta):
    """(loss, w (18,)) of one engine sweep over ``freqs`` (scale 1 / |freqs|), as bench.gpu_parity."""
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.Problem import _coeffs18
    eng = p.engine(freqs.size)
    c = _coeffs18(p._transform(), torch.as_tensor(theta)).detach().numpy()
    eng.set_coefficients(c)
    dev = eng.device
    w = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
    loss = torch.zeros(1, dtype=torch.float64, device=dev)
    eng.sweep(torch.as_tensor(freqs, device=dev), _native.LOSS_MSE_LOG_AFC,
              ref=torch.view_as_real(torch.as_tensor(ref.astype(np.complex128), device=dev)), scale=1.0 / freqs.size,
              loss=loss, w=torch.view_as_real(w))
    return float(loss.item()) / freqs.size, eng.expand(w).cpu().numpy()


def _check_set(name, p, T, sel, theta):
    from oracle.plate_oracle import coeffs18_jacobian
    f, ref = T["freqs"][sel], T["ref"][sel]
    loss, w = _gpu_partials(p, f, ref, theta)
    wt = T["w_true"][sel].sum(0) / sel.size
    wo = T["w_oracle"][sel].sum(0) / sel.size
    lt = T["term_true"][sel].mean()
    lo = T["term_oracle"][sel].mean()
    J = coeffs18_jacobian("orthotropic", p.geometry.height, theta)
    gt, gg, go = (np.real(v @ J) for v in (wt, w, wo))
    e = dict(w_gpu=_wrel(w, wt), w_oracle=_wrel(wo, wt), loss_gpu=abs(loss / lt - 1), loss_oracle=abs(lo / lt - 1),
             grad_gpu=_wrel(gg, gt), grad_oracle=_wrel(go, gt), n=sel.size)
    report(name, **e)
    assert e["w_gpu"] <= W_RTOL, e
    assert e["grad_gpu"] <= W_RTOL, e
    assert e["loss_gpu"] <= LOSS_RTOL, e
    return e


@pytest.fixture(scope="module")
def c3_fresh():
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    yield p
    p._engine = None
    del p
    gc.collect()
    torch.cuda.empty_cache()


def test_c3_full_sweep_gradient_vs_truth(c3_fresh):
    """The bench's loss + gradient over all 4,096 frequencies (2 lanes x 2,048), then the bench's
    2,048-frequency parity subsample and the 32 fixture frequencies of c3_truth.npz, on the same engine."""
    T = _truth()
    p = c3_fresh
    assert p.mat_size == 19353 and int(T["n_sweep"]) == 4096 and T["freqs"].size == 4096
    theta = np.asarray(T["theta"])
    assert np.allclose(theta, p.parameters * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1])), rtol=1e-15)
    every = np.arange(4096)
    _check_set("c3_grad_truth_4096", p, T, every, theta)
    eng = p.engine()
    assert eng.n_lanes == 2 and eng.max_batch == 2048
    bench_sample = np.linspace(0, 4095, 2048).round().astype(int)       # bench.cpu_baseline, 16 cores
    _check_set("c3_grad_truth_bench2048", p, T, bench_sample, theta)
    fixture = np.load(os.path.join(GOLDEN, "c3_truth.npz"))["index"]
    _check_set("c3_grad_truth_fixture32", p, T, np.asarray(fixture), theta)
    # and through the public API (autograd through the material transform): the theta gradient
    x = torch.tensor(theta, requires_grad=True)
    val = p.getLossFunction(T["freqs"], T["ref"].astype(np.complex128), "MSE_LOG_AFC")(x)
    val.backward()
    assert not np.any(p.engine().last_flags)
    from oracle.plate_oracle import coeffs18_jacobian
    gt = np.real(T["w_true"].sum(0) / 4096 @ coeffs18_jacobian("orthotropic", p.geometry.height, theta))
    go = np.real(T["w_oracle"].sum(0) / 4096 @ coeffs18_jacobian("orthotropic", p.geometry.height, theta))
    report("c3_grad_truth_api", grad_gpu=_wrel(x.grad.numpy(), gt), grad_oracle=_wrel(go, gt),
           loss_gpu=abs(val.item() / T["term_true"].mean() - 1))
    assert _wrel(x.grad.numpy(), gt) <= W_RTOL


def test_c4_rank_block_at_c3_size():
    """C4's per-rank workload: a fresh C3 problem whose first sweep is rank 2's 512-frequency block of
    the 8-GPU strong-scaling run -- the narrow-sweep engine -- fr against the extended-precision fixture,
    loss and gradient against the truth."""
    from plate_inverse_problem_amd.distributed import shard_range
    T = _truth()
    F = np.load(os.path.join(GOLDEN, "c3_truth.npz"))
    lo, hi = shard_range(4096, 2, 8)
    assert (lo, hi) == (1024, 1536) and lo <= 1179 < hi
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    try:
        theta = np.asarray(T["theta"])
        sel = np.arange(lo, hi)
        e = _check_set("c4_rank2_grad_truth", p, T, sel, theta)
        eng = p.engine()
        assert eng.n_lanes == 2 and eng.max_batch == 256       # two lanes of 256 (Problem._lanes_for)
        assert eng.leaf_size_for(512) == 2000 and eng.sym is eng._syms[2000]
        assert eng.stats["n_levels"] < 38          # the shallow tree, not the deep one
        # fr at the fixture frequencies inside the block (forward sweep on the same engine)
        inside = (F["index"] >= lo) & (F["index"] < hi)
        assert inside.sum() >= 5
        fr = p.solveForward(F["freqs"][inside])
        assert p.engine() is eng
        err = np.abs(fr / F["fr_true"][inside] - 1)
        err_o = np.abs(F["fr_oracle"][inside] / F["fr_true"][inside] - 1)     # the refined oracle, same frequencies
        report("c4_rank2_fr_vs_truth", gpu_max=err.max(), oracle_max=err_o.max(), n=int(inside.sum()),
               **{k: v for k, v in e.items() if k != "n"})
        # absolute FR_RTOL_C3 at every fixture frequency (round 4 needed max(1e-7, 2x the oracle's error) for the
        # leaf-200 ordering's 1.04e-7 at 200 Hz, since round 5 at 1,000; the compensated residual of the functional correction makes the
        # corrected fr independent of the factorisation's rounding order)
        assert np.all(err < FR_RTOL_C3), (err, err_o)
    finally:
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()
