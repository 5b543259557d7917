"""Loss functions of the hot path as autograd Functions over the HIP kernels (no ATen compute)."""
import torch

from . import kernels as K


class _MSELoss(torch.autograd.Function):
    """F.mse_loss(a, b) with mean reduction (autencoder_lightning_base.py:68,82)."""

    @staticmethod
    def forward(ctx, a, b):
        a_, b_ = a.contiguous(), b.contiguous()
        sq = torch.zeros(1, device=a.device, dtype=torch.float64)
        K.mse_fwd(a_, b_, sq)
        out = torch.empty((), device=a.device)
        K.mse_finalize(sq, a.numel(), out)
        ctx.save_for_backward(a_, b_)
        ctx.b_needs = b.requires_grad
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        ga = torch.empty_like(a)
        K.mse_bwd(a, b, g.reshape(1).contiguous(), ga)
        gb = None
        if ctx.b_needs:
            gb = torch.empty_like(b)
            K.mse_bwd(b, a, g.reshape(1).contiguous(), gb)
        return ga, gb


def mse_loss(a, b):
    return _MSELoss.apply(a, b)


class _AddScalars(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        out = torch.empty((), device=a.device)
        K.scalar_add(a.reshape(1).contiguous(), b.reshape(1).contiguous(), out)
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g


def add_scalars(a, b):
    return _AddScalars.apply(a, b)
