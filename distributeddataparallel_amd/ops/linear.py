"""Bias-free linear layer on the own transformer GEMM (``csrc/kernels/gemm.hip``) for the
Llama-3-8B config of BASELINE.json: the forward ``y = x·Wᵀ`` (optionally ``residual + x·Wᵀ``, the
pre-norm block's skip connection added in the GEMM epilogue instead of a separate add pass) runs
on the LDS-DMA MFMA kernel; the backward's ``dX = dY·W`` and ``dW = dYᵀ·X`` stay on hipBLASLt.

The module structure is untouched (``nn.Linear`` parameters), so state_dicts and DDP buckets are
the same as the eager model's.

``XDDP_OWN_GEMM`` selects where the own GEMM runs: ``1`` every supported projection (forward
epilogues included), ``bwd`` (default) only the backward GEMM that carries a fused epilogue
hipBLASLt cannot do (the ViT MLP's dGELU + bias gradient), ``0`` nowhere. On one MI355X the own
kernel reaches 0.80-0.93x hipBLASLt's plain-GEMM speed on the transformer shapes
(``profiles/r3_gemm_nt_vs_hipblaslt.txt``), so forward projections stay on hipBLASLt, whose
beta = 1 residual accumulate is free, unless asked for.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["linear", "own_gemm_ok", "own_gemm_mode"]


def own_gemm_mode() -> str:
    """``XDDP_OWN_GEMM``: ``"1"`` (all), ``"bwd"`` (fused-epilogue backward GEMMs only, default) or ``"0"``."""
    v = os.environ.get("XDDP_OWN_GEMM", "bwd")
    return v if v in ("0", "1", "bwd") else "bwd"


def own_gemm_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if own_gemm_mode() != "1" or torch.is_autocast_enabled():
        return False
    N, K = weight.shape
    return (x.is_cuda and x.dtype == torch.bfloat16 and weight.dtype == torch.bfloat16 and K % 64 == 0
            and N % 128 == 0 and x.shape[-1] == K and weight.is_contiguous())


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, residual):
        C = load()
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if x2.stride(0) != shape[-1] or x2.stride(-1) != 1 or x2.data_ptr() % 16:
            x2 = x2.contiguous()
        if residual is None:
            y = C.gemm_nt(x2, weight)[0]
        else:
            r2 = residual.reshape(-1, weight.shape[0])
            y = C.gemm_nt(x2, weight, None, 3, r2)[0]
        ctx.save_for_backward(x2, weight)
        ctx.shape, ctx.has_res = shape, residual is not None
        return y.view(*shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[0])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.mm(dy2, weight).view(ctx.shape)
        if ctx.needs_input_grad[1]:
            dw = torch.mm(dy2.t(), x2)
        dres = dy if ctx.has_res and ctx.needs_input_grad[2] else None
        return dx, dw, dres


def linear(x: torch.Tensor, weight: torch.Tensor, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``x·Wᵀ`` (+ ``residual``) — the own GEMM when the shapes allow it, else ``F.linear``."""
    if own_gemm_ok(x, weight) and (residual is None or (residual.shape[:-1] == x.shape[:-1]
                                                        and residual.dtype == torch.bfloat16
                                                        and residual.is_contiguous())):
        return _Linear.apply(x, weight, residual)
    y = F.linear(x, weight)
    return y if residual is None else residual + y
