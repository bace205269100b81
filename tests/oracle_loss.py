"""The oracle's loss + adjoint gradient as a torch autograd function (drives this build's optimisers
the way the GPU loss does, for optimiser-trajectory comparisons)."""
import numpy as np
import torch


def oracle_loss_fn(orc, freqs, ref, loss_type, scaling=None):
    from oracle.plate_oracle import loss_and_grad

    class _L(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            val, g = loss_and_grad(orc, freqs, ref, loss_type, x.detach().cpu().numpy(), scaling=scaling)
            ctx.save_for_backward(torch.as_tensor(g))
            return torch.tensor(val, dtype=torch.float64)

        @staticmethod
        def backward(ctx, go):
            (g,) = ctx.saved_tensors
            return g * go

    return lambda x: _L.apply(torch.as_tensor(np.asarray(x, dtype=np.float64) if not isinstance(x, torch.Tensor)
                                              else x, dtype=torch.float64))
