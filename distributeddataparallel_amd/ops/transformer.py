"""Fused rotary embedding and SwiGLU for the Llama config (``csrc/kernels/transformer.hip``).

``rope(x, cos, sin)`` rotates ``x: [B, S, H, Dh]`` (the layout the q/k projections produce,
before the head transpose) in one pass; its backward is the inverse rotation of the gradient.
``swiglu(a, b) = silu(a) * b`` in one pass; backward recomputes ``sigmoid(a)`` and writes both
input gradients in one pass. Shapes the kernels do not cover (CPU, non-contiguous, sizes not a
multiple of 8) take the equivalent PyTorch path.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["rope", "swiglu", "rope_reference"]


def rope_reference(x, cos, sin):
    """PyTorch reference: rotate (even, odd) pairs of the last dim of ``x: [B, S, H, Dh]``."""
    S = x.shape[1]
    c, s = cos[:S][None, :, None, :], sin[:S][None, :, None, :]
    x1, x2 = x[..., 0::2].float(), x[..., 1::2].float()
    return torch.stack([x1 * c - x2 * s, x1 * s + x2 * c], dim=-1).flatten(-2).to(x.dtype)


class _Rope(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin):
        ctx.save_for_backward(cos, sin)
        return load().rope(x, cos, sin, False)

    @staticmethod
    def backward(ctx, dy):
        cos, sin = ctx.saved_tensors
        return load().rope(dy.contiguous(), cos, sin, True), None, None


class _SwiGLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return load().swiglu_forward(a, b)

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        da, db = load().swiglu_backward(g.contiguous(), a, b)
        return da, db


def _vec_ok(*ts):
    return all(t.is_cuda and t.is_contiguous() and t.numel() % 8 == 0 and t.data_ptr() % 16 == 0 and
               t.dtype in (torch.bfloat16, torch.float16, torch.float32) for t in ts)


def rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Rotary embedding of ``x: [B, S, H, Dh]`` with fp32 tables ``cos, sin: [>= S, Dh/2]``."""
    if (_vec_ok(x) and x.dim() == 4 and x.shape[-1] % 8 == 0 and cos.is_cuda and cos.dtype == torch.float32
            and cos.is_contiguous() and sin.is_contiguous()):
        return _Rope.apply(x, cos, sin)
    return rope_reference(x, cos, sin)


def swiglu(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``silu(a) * b`` (the Llama MLP gate)."""
    if _vec_ok(a, b) and a.shape == b.shape and a.dtype == b.dtype:
        return _SwiGLU.apply(a, b)
    return F.silu(a) * b
