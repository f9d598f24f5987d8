"""LayerNorm / RMSNorm on xddp's wave-per-row HIP kernels (ViT-L/16, Llama-3 configs).

``FusedLayerNorm`` subclasses ``nn.LayerNorm`` and ``FusedRMSNorm`` mirrors ``nn.RMSNorm``
(same parameter names, so checkpoints and DDP bucket layouts are unchanged). Shapes the
kernels do not cover (last dim % 8 != 0 or > 8192, CPU tensors) take the PyTorch path.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import load

__all__ = ["FusedLayerNorm", "FusedRMSNorm", "layer_norm", "rms_norm", "rms_norm_with_skip"]


class _LN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, rms):
        C = load()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        y, mean, rstd, _ = C.ln_forward(x2, weight, bias, eps, rms)
        ctx.rms = rms
        ctx.save_for_backward(x2, weight, mean if not rms else None, rstd)
        ctx.shape = shape
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        C = load()
        x2, weight, mean, rstd = ctx.saved_tensors
        dx, dg, db, _, _ = C.ln_backward(dy.reshape(x2.shape), x2, weight, mean, rstd, ctx.rms,
                                   ctx.needs_input_grad[1], ctx.needs_input_grad[2])
        return dx.view(ctx.shape), dg, (db if not ctx.rms else None), None, None


class _RMSSkip(torch.autograd.Function):
    """RMSNorm whose input is also the block's skip connection: returns (y, skip), skip an alias of
    x. Autograd hands this node both gradients at once, so the skip connection's gradient is added
    inside the norm's backward kernel (``ln_backward(..., res=)``) instead of by a separate add
    pass over the residual stream (two per Llama block)."""

    @staticmethod
    def forward(ctx, x, weight, eps):
        C = load()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        y, _, rstd, _ = C.ln_forward(x2, weight, None, eps, True)
        ctx.save_for_backward(x2, weight, rstd)
        ctx.shape = shape
        return y.view(shape), x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dskip):
        C = load()
        x2, weight, rstd = ctx.saved_tensors
        if dy is None:
            return dskip, None, None
        res = dskip.reshape(x2.shape) if dskip is not None else None
        dx, dg, _, _, _ = C.ln_backward(dy.reshape(x2.shape), x2, weight, None, rstd, True,
                                        ctx.needs_input_grad[1], False, res)
        return dx.view(ctx.shape), dg, None


def rms_norm_with_skip(x, normalized_shape, weight=None, eps=1e-6):
    """``(rms_norm(x), x)`` for a pre-norm block whose skip connection is ``x``: on the fused path
    the skip's gradient is summed inside the norm's backward (see :class:`_RMSSkip`)."""
    d = x.shape[-1]
    if len(normalized_shape) == 1 and _ok(x, d) and weight is not None and x.dtype == weight.dtype:
        return _RMSSkip.apply(x, weight, float(eps))
    return rms_norm(x, normalized_shape, weight, eps), x


def _ok(x, d):
    return x.is_cuda and d % 8 == 0 and d <= 8192 and x.dtype in (torch.bfloat16, torch.float16, torch.float32)


def layer_norm(x, normalized_shape, weight=None, bias=None, eps=1e-5):
    d = x.shape[-1]
    if len(normalized_shape) == 1 and _ok(x, d):
        return _LN.apply(x, weight, bias, float(eps), False)
    return F.layer_norm(x, normalized_shape, weight, bias, eps)


def rms_norm(x, normalized_shape, weight=None, eps=1e-6):
    d = x.shape[-1]
    if len(normalized_shape) == 1 and _ok(x, d):
        return _LN.apply(x, weight, None, float(eps), True)
    var = x.float().pow(2).mean(-1, keepdim=True)
    y = (x.float() * torch.rsqrt(var + eps)).to(x.dtype)
    return y * weight if weight is not None else y


class FusedLayerNorm(nn.LayerNorm):
    def forward(self, x):
        return layer_norm(x, self.normalized_shape, self.weight, self.bias, self.eps)


class FusedRMSNorm(nn.Module):
    def __init__(self, normalized_shape, eps: float = 1e-6, elementwise_affine: bool = True, device=None, dtype=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = tuple(normalized_shape)
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(self.normalized_shape, device=device, dtype=dtype)) \
            if elementwise_affine else None

    def forward(self, x):
        return rms_norm(x, self.normalized_shape, self.weight, self.eps)

    def forward_with_skip(self, x):
        """``(self(x), x)`` with the skip connection's gradient added in this norm's backward."""
        return rms_norm_with_skip(x, self.normalized_shape, self.weight, self.eps)

    def extra_repr(self):
        return f"{self.normalized_shape}, eps={self.eps}"
