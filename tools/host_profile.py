import cProfile, pstats, sys, time, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from bench import build_problem
p = build_problem(25, torch.device("cuda", 0))
freqs = np.linspace(40.0, 600.0, int(os.environ.get("HP_FREQS", "4096")))
th = p.parameters.copy()
ref = p.solveForward(freqs, th)
loss_fn = p.getLossFunction(freqs, ref, "MSE_LOG_AFC")
theta = th * 1.1
def step():
    x = torch.tensor(theta, requires_grad=True)
    v = loss_fn(x); v.backward(); return v.item(), x.grad
for _ in range(2): step()
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(5): step()
pr.disable()
torch.cuda.synchronize()
print("ms/step", (time.perf_counter()-t0)/5*1e3)
pstats.Stats(pr).sort_stats(os.environ.get("HP_SORT", "tottime")).print_stats(30)
