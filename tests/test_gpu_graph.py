"""GPU: sweep graphs (PFR_GRAPH, api.cpp pfr_sweep).  A loss + gradient step repeated with the same arguments is
captured into a hipGraph on its second call and replayed afterwards; the replay runs the same kernels with the same
arguments, so loss, gradient and backward errors must EQUAL the direct launches' bit for bit.  A step at a new
theta (pfr_set_rhs in between: a new solver state) must leave the graph and run directly, and the same theta
again must be captured again.  Workload: C4's per-rank block (512 frequencies of the C3 sweep, the one with the
resonance), the loop an optimiser or the bench runs (Problem.getLossFunction + backward)."""
import gc
import os

import numpy as np
import pytest
import torch

from helpers import make_problem, report

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _steps(monkeypatch, graph, thetas):
    from plate_inverse_problem_amd.distributed import shard_range
    monkeypatch.setenv("PFR_GRAPH", graph)
    T = np.load(os.path.join(GOLDEN, "c3_grad_truth.npz"))
    lo, hi = shard_range(4096, 2, 8)
    sel = np.arange(lo, hi)
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    try:
        fn = p.getLossFunction(T["freqs"][sel], T["ref"][sel], "MSE_LOG_AFC")
        out = []
        for th in thetas:
            x = torch.tensor(th, requires_grad=True)
            v = fn(x)
            v.backward()
            eng = p.engine()
            out.append((v.item(), x.grad.numpy().copy(), eng.last_berr.cpu().numpy().copy()))
        eng = p.engine()
        return out, sum(sv.graph_launches() for sv in eng.solvers), eng.n_lanes
    finally:
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()


def test_graph_replay_bitwise_and_state_changes(monkeypatch):
    T = np.load(os.path.join(GOLDEN, "c3_grad_truth.npz"))
    t0 = np.asarray(T["theta"], dtype=np.float64)
    t1 = t0 * (1 + 0.01 * np.arange(1, t0.size + 1))
    # t0 x4: direct, captured, replayed, replayed; t1 x3: direct (new rhs scale), captured, replayed; t0: direct
    thetas = [t0, t0, t0, t0, t1, t1, t1, t0]
    direct, n0, lanes = _steps(monkeypatch, "0", thetas)
    graph, n1, lanes1 = _steps(monkeypatch, "1", thetas)
    assert n0 == 0 and lanes == lanes1
    assert n1 == 5 * lanes, n1
    dl = max(abs(g[0] - d[0]) for g, d in zip(graph, direct))
    dw = max(float(np.max(np.abs(g[1] - d[1]))) for g, d in zip(graph, direct))
    db = max(float(np.nanmax(np.abs(g[2] - d[2]))) for g, d in zip(graph, direct))
    report("graph_replay_vs_direct", loss_diff=dl, grad_diff=dw, berr_diff=db, graph_launches=n1, lanes=lanes)
    for k, (g, d) in enumerate(zip(graph, direct)):
        assert g[0] == d[0], (k, g[0], d[0])
        assert np.array_equal(g[1], d[1]), k
        assert np.array_equal(np.isnan(g[2]), np.isnan(d[2])) and np.array_equal(np.nan_to_num(g[2]),
                                                                                  np.nan_to_num(d[2])), k
    # the steps at one theta agree among themselves (replays of one graph and the direct run before them)
    assert graph[0][0] == graph[3][0] and np.array_equal(graph[0][1], graph[3][1])
    assert graph[4][0] != graph[0][0]


def test_graph_two_lanes_repeated_steps(monkeypatch):
    """C3's 4,096 frequencies on two lanes (two solvers, two host threads, each capturing and replaying its own
    graph): twelve steps at one theta -- every step's loss and gradient equal to the first (direct) step's, no
    frequency flagged by the on-device backward-error checks."""
    import bench
    monkeypatch.setenv("PFR_GRAPH", "1")
    p = bench.build_problem(25, torch.device("cuda", 0))
    try:
        th0 = p.parameters.copy()
        freqs = np.linspace(40.0, 600.0, 4096)
        ref = p.solveForward(freqs, th0)
        fn = p.getLossFunction(freqs, ref, "MSE_LOG_AFC")
        theta = th0 * (1 + np.array([0.1, 0.1, 0.2, 0.1, 0.1]))
        vals, grads, nflag = [], [], []
        for _ in range(12):
            x = torch.tensor(theta, requires_grad=True)
            v = fn(x)
            v.backward()
            eng = p.engine()
            vals.append(v.item())
            grads.append(x.grad.numpy().copy())
            nflag.append(int(np.count_nonzero(eng.last_flags)))
        n_graph = sum(sv.graph_launches() for sv in eng.solvers)
        report("graph_two_lanes", lanes=eng.n_lanes, graph_launches=n_graph, flagged=max(nflag),
               loss_spread=max(vals) - min(vals))
        assert eng.n_lanes == 2 and n_graph == 2 * 11      # step 1 direct (new theta), 2 captured, 3-12 replayed
        assert max(nflag) == 0, nflag
        for k in range(1, 12):
            assert vals[k] == vals[0] and np.array_equal(grads[k], grads[0]), k
    finally:
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()


def test_fresh_sweep_initialises_its_outputs():
    """pfr_sweep_fresh (the loss step's sweeps): the loss / w slots, flags and backward errors are initialised by the
    sweep itself -- with the step buffers poisoned beforehand, the loss, gradient partials and backward errors equal
    those of the accumulating pfr_sweep into freshly zeroed / NaN-filled buffers, bit for bit."""
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.distributed import shard_range
    from plate_inverse_problem_amd.Problem import _coeffs18
    T = np.load(os.path.join(GOLDEN, "c3_grad_truth.npz"))
    lo, hi = shard_range(4096, 2, 8)
    sel = np.arange(lo, hi)
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    try:
        eng = p.engine(sel.size)
        eng.set_coefficients(_coeffs18(p._transform(), torch.as_tensor(T["theta"])).detach().numpy())
        dev = eng.device
        f = torch.as_tensor(T["freqs"][sel], device=dev)
        ref = torch.view_as_real(torch.as_tensor(T["ref"][sel].astype(np.complex128), device=dev))
        eng.loss_step(f, _native.LOSS_MSE_LOG_AFC, ref, 1.0 / sel.size)
        for buf in eng._step_bufs.values():            # poison every step buffer
            buf[0].fill_(1e300)
            buf[2].fill_(7)
            buf[3].fill_(123.0)
        lsum, w, flags, nflag = eng.loss_step(f, _native.LOSS_MSE_LOG_AFC, ref, 1.0 / sel.size)
        berr_fresh = eng.last_berr.cpu().numpy().copy()
        loss = torch.zeros(1, dtype=torch.float64, device=dev)
        wv = torch.zeros(eng.n_stiff, dtype=torch.complex128, device=dev)
        fl = torch.zeros(sel.size, dtype=torch.int32, device=dev)
        berr = torch.full((sel.size, 2), float("nan"), dtype=torch.float64, device=dev)
        eng.sweep(f, _native.LOSS_MSE_LOG_AFC, ref=ref, scale=1.0 / sel.size, loss=loss, w=torch.view_as_real(wv),
                  flags=fl, berr=berr)
        w_acc = eng.expand(wv).cpu().numpy()
        report("fresh_sweep", loss_fresh=lsum, loss_acc=float(loss.item()), nflag=nflag)
        assert nflag == 0 and int(fl.count_nonzero()) == 0 and int(flags.count_nonzero()) == 0
        assert lsum == float(loss.item())
        assert np.array_equal(w, w_acc)
        b = berr.cpu().numpy()
        assert np.array_equal(np.isnan(berr_fresh), np.isnan(b)) and np.array_equal(np.nan_to_num(berr_fresh),
                                                                                    np.nan_to_num(b))
    finally:
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()


def test_jet_loss_is_one_node_and_matches_the_chain():
    """getLossFunction on a jet-transform material (Problem._JetSweepLoss): one autograd node from params to the
    loss, and loss and gradient EQUAL the three-node chain params * scaling -> _Coeffs -> _SweepLoss on the same
    engine, bit for bit (with a parameter scaling, as the reference's scaling_params)."""
    from plate_inverse_problem_amd import _native
    from plate_inverse_problem_amd.distributed import shard_range
    from plate_inverse_problem_amd.Problem import _SweepLoss
    T = np.load(os.path.join(GOLDEN, "c3_grad_truth.npz"))
    lo, hi = shard_range(4096, 2, 8)
    sel = np.arange(lo, hi)
    p = make_problem("orthotropic", ny=25, device="cuda:0")
    try:
        scal = np.array([1.0, 2.0, 0.5, 1.0, 1.0])
        th = np.asarray(T["theta"]) / scal
        fn = p.getLossFunction(T["freqs"][sel], T["ref"][sel], "MSE_LOG_AFC", scaling_params=scal)
        x = torch.tensor(th, requires_grad=True)
        v = fn(x)
        assert type(v.grad_fn).__name__ == "_JetSweepLossBackward"
        assert [type(f).__name__ for f, _ in v.grad_fn.next_functions if f is not None] == ["AccumulateGrad"]
        v.backward()
        y = torch.tensor(th, requires_grad=True)
        c = p._coeffs(p._transform(), y.to(torch.float64).cpu() * torch.as_tensor(scal))
        u = _SweepLoss.apply(c, p.engine(sel.size), p._freqs(T["freqs"][sel]),
                             torch.as_tensor(T["ref"][sel].astype(np.complex128), device=p.device),
                             _native.LOSS_IDS["MSE_LOG_AFC"], sel.size, None)
        u.backward()
        report("jet_loss_node", loss=v.item(), grad_diff=float(np.max(np.abs(x.grad.numpy() - y.grad.numpy()))))
        assert v.item() == u.item()
        assert np.array_equal(x.grad.numpy(), y.grad.numpy())
    finally:
        p._engine = None
        del p
        gc.collect()
        torch.cuda.empty_cache()
