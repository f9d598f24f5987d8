"""Flash attention on gfx950 MFMA kernels (``csrc/kernels/flash_attn.hip``) for the ViT-L/16 and
Llama-3-8B configs of BASELINE.json.

Inputs and output are ``[B, S, H, D]`` (the projection's own layout: q/k/v are views of the
projection outputs and the output reshapes to ``[B, S, H·D]`` for the output projection without a
copy). Grouped-query attention: ``k``/``v`` may have fewer heads than ``q``. bf16, D in {64, 128}.

``XDDP_FLASH_ATTN=0`` sends every call to ``F.scaled_dot_product_attention`` (A/B and parity).
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["flash_attention", "flash_supported"]


def flash_supported(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor) -> bool:
    if os.environ.get("XDDP_FLASH_ATTN", "1") == "0":
        return False
    D = q.shape[-1]
    ok = (q.is_cuda and q.dtype == torch.bfloat16 and k.dtype == torch.bfloat16 and v.dtype == torch.bfloat16
          and q.dim() == 4 and D in (64, 128) and k.shape[-1] == D and v.shape == k.shape
          and q.shape[2] % k.shape[2] == 0)
    if not ok:
        return False
    for t in (q, k, v):
        if t.stride(-1) != 1 or any(s % 8 for s in t.stride()[:3]) or t.data_ptr() % 16:
            return False
    return True


class _FlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal: bool, scale: float):
        o, lse = load().flash_attn_forward(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.causal, ctx.scale = causal, scale
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        if do.stride(-1) != 1 or any(s % 8 for s in do.stride()[:3]):
            do = do.contiguous()
        dq, dk, dv = load().flash_attn_backward(do, q, k, v, o, lse, ctx.causal, ctx.scale)
        return dq, dk, dv, None, None


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, causal: bool = False,
                    scale: float | None = None) -> torch.Tensor:
    """softmax(q kᵀ · scale [+ causal mask]) v over [B, S, H, D] tensors; returns [B, S, H, D]."""
    scale = 1.0 / math.sqrt(q.shape[-1]) if scale is None else scale
    if flash_supported(q, k, v):
        return _FlashAttn.apply(q, k, v, causal, scale)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), is_causal=causal,
                                       scale=scale, enable_gqa=k.shape[2] != q.shape[2])
    return o.transpose(1, 2)
