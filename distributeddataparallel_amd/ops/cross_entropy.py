"""Softmax cross-entropy on xddp's HIP kernels (``csrc/kernels/cross_entropy.hip``) for the
Llama-3-8B LM head of BASELINE.json config 5: bf16 logits [rows, vocab], fp32 math, mean over
the non-ignored rows — ``F.cross_entropy(logits.float(), target)`` without the 2.1 GB fp32 copy
of the logits, its zero-filled fp32 gradient and the casts (one read of the logits forward, one
read + one bf16 write backward). CPU tensors and other dtypes / shapes fall back to torch.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["cross_entropy"]


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        C = load()
        loss_rows, lse = C.cross_entropy_forward(logits, target, ignore_index)
        count = (target != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, target, lse, count)
        ctx.ignore_index = ignore_index
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, count = ctx.saved_tensors
        gscale = (g.to(torch.float32) / count).reshape(1).contiguous()
        d = load().cross_entropy_backward(logits, target, lse, gscale, ctx.ignore_index)
        return d, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy of ``logits`` [rows, classes] against ``target`` [rows]; bf16
    CUDA logits with a class count divisible by 8 run the fused kernels, anything else
    ``F.cross_entropy`` on the fp32 upcast."""
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2 and logits.size(1) % 8 == 0
            and target.dtype == torch.long and target.dim() == 1):
        return _CrossEntropy.apply(logits.contiguous(), target.contiguous(), ignore_index)
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
