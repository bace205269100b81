"""The oracle's loss + adjoint gradient as a torch autograd function (drives this build's optimisers
the way the GPU loss does, for optimiser-trajectory comparisons)."""
import numpy as np
import torch


def _parallel_loss_and_grad(orc, freqs, ref, loss_type, theta, scaling, n_workers):
    """loss_and_grad with the frequency partials from a process pool (large meshes)."""
    from oracle.plate_oracle import coeffs18_jacobian, parallel_partials
    theta = np.asarray(theta, dtype=np.float64)
    s = np.ones_like(theta) if scaling is None else np.asarray(scaling, dtype=np.float64)
    phys = theta * s
    loss_sum, w, _ = parallel_partials(orc, freqs, ref, loss_type, phys, n_workers=n_workers)
    J = coeffs18_jacobian(orc.atype, orc.h, phys, orc.angles)
    return loss_sum / np.asarray(freqs).size, np.real(w @ J) * s


def oracle_loss_fn(orc, freqs, ref, loss_type, scaling=None, n_workers=None):
    from oracle.plate_oracle import loss_and_grad

    class _L(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            xn = x.detach().cpu().numpy()
            if n_workers:
                val, g = _parallel_loss_and_grad(orc, freqs, ref, loss_type, xn, scaling, n_workers)
            else:
                val, g = loss_and_grad(orc, freqs, ref, loss_type, xn, scaling=scaling)
            ctx.save_for_backward(torch.as_tensor(g))
            return torch.tensor(val, dtype=torch.float64)

        @staticmethod
        def backward(ctx, go):
            (g,) = ctx.saved_tensors
            return g * go

    return lambda x: _L.apply(torch.as_tensor(np.asarray(x, dtype=np.float64) if not isinstance(x, torch.Tensor)
                                              else x, dtype=torch.float64))
