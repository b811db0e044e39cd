"""Drop-in for utils/ops.py: clamp with one-sided pass-through gradient on HIP.

Low_bound  utils/ops.py:28-41  fwd clamp(min=b); bwd g * ((x >= b) | (g < 0))
Up_bound   utils/ops.py:43-56  fwd clamp(max=b); bwd g * ((x <= b) | (g > 0))
Round_STE  utils/ops.py:8-15

The attack hot path fuses these into its kernels (ica_attack_prologue / ica_attack_loss /
ica_attack_adam); these autograd Functions serve user code that composes them directly.
"""
from __future__ import annotations

import torch


class Low_bound(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, lower_bound=1e-6):
        ctx.save_for_backward(x)
        ctx.lower_bound = lower_bound
        return torch.clamp(x, min=lower_bound)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * ((x >= ctx.lower_bound) | (g < 0.0)).to(g.dtype), None


class Up_bound(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, up_bound=1.0):
        ctx.save_for_backward(x)
        ctx.up_bound = up_bound
        return torch.clamp(x, max=up_bound)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return g * ((x <= ctx.up_bound) | (g > 0.0)).to(g.dtype), None


class Round_STE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.round()

    @staticmethod
    def backward(ctx, g):
        return g


from ..codec import GDN  # noqa: E402,F401  (GDN parameters; the normalisation runs fused)
