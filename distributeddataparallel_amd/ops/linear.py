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
import weakref
from typing import Optional

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["linear", "multi_linear", "own_gemm_ok", "own_gemm_mode", "set_grad_targets", "clear_grad_targets"]

# weight -> the tensor its gradient should be written into (DDP with gradient_as_bucket_view
# registers each parameter's view of its bucket, ``DistributedDataParallel._pre_forward``)
# (keyed by id: a WeakKeyDictionary would compare tensor keys with elementwise ==). Both the
# parameter and the target are held weakly: the DDP object owns the bucket views, so a deleted
# DDP (or a rebuilt bucket layout) leaves only dead entries behind, never live bucket memory.
_GRAD_TARGETS: dict = {}  # id(param) -> (weakref(param), weakref(target))


def _autocast_on(t: torch.Tensor) -> bool:
    """Autocast active for ``t``'s device type: the custom Functions below have no
    custom_fwd/custom_bwd casts, so under autocast every path here defers to ``F.linear``."""
    return torch.is_autocast_enabled(t.device.type)


def set_grad_targets(params, targets) -> None:
    """Register ``targets[i]`` (same shape / dtype / device, dense) as where the weight gradient
    of ``params[i]`` is written when the parameter holds no gradient yet: the backward GEMM writes
    ``dW`` straight into it and hands autograd a fresh alias, which ``AccumulateGrad`` adopts as
    ``.grad`` — so DDP finds the gradient already in its bucket instead of copying it there (one
    read + one write of every weight gradient per step; 16 GB for Llama-3-8B)."""
    for p, t in zip(params, targets):
        if t is not None and t.shape == p.shape and t.dtype == p.dtype and t.device == p.device and t.is_contiguous():
            _GRAD_TARGETS[id(p)] = (weakref.ref(p), weakref.ref(t))
        else:
            _GRAD_TARGETS.pop(id(p), None)


def _dw(dy2: torch.Tensor, x2: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``dW = dY2ᵀ·X2`` for weight ``w`` — into its registered target when ``w`` has no gradient
    yet (the first contribution of this backward), returned as a fresh alias of it."""
    e = _GRAD_TARGETS.pop(id(w), None)  # one claim per registration: a weight used twice in a
    t = e[1]() if e is not None and e[0]() is w else None  # forward gets one target write
    if t is not None and w.grad is None and not torch.is_grad_enabled():
        torch.mm(dy2.t(), x2, out=t)
        return t.view(t.shape)
    return torch.mm(dy2.t(), x2)


def own_gemm_mode() -> str:
    """``XDDP_OWN_GEMM``: ``"1"`` (all), ``"bwd"`` (fused-epilogue backward GEMMs only, default) or ``"0"``."""
    v = os.environ.get("XDDP_OWN_GEMM", "bwd")
    return v if v in ("0", "1", "bwd") else "bwd"


def clear_grad_targets(params) -> None:
    """Drop the registrations of ``params`` (a DDP being torn down or rebuilt)."""
    for p in params:
        _GRAD_TARGETS.pop(id(p), None)


def own_gemm_ok(x: torch.Tensor, weight: torch.Tensor) -> bool:
    if own_gemm_mode() != "1" or _autocast_on(x):
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
    """``x·Wᵀ`` (+ ``residual``) — the own GEMM when the shapes allow it, else the library GEMM,
    with the residual as its beta = 1 accumulate operand (``addmm``: one GEMM, one rounding, no
    separate add pass over the residual stream)."""
    if own_gemm_ok(x, weight) and (residual is None or (residual.shape[:-1] == x.shape[:-1]
                                                        and residual.dtype == torch.bfloat16
                                                        and residual.is_contiguous())):
        return _Linear.apply(x, weight, residual)
    if residual is not None and (residual.shape[:-1] != x.shape[:-1] or residual.dtype != x.dtype):
        return residual + F.linear(x, weight)
    if weight.dim() != 2 or x.dtype != weight.dtype or _autocast_on(x):
        y = F.linear(x, weight)
        return y if residual is None else residual + y
    return _LinearBlas.apply(x, weight, residual)


class _LinearBlas(torch.autograd.Function):
    """``x·Wᵀ`` (+ ``residual`` as the GEMM's beta = 1 operand) on the library GEMM; the backward
    writes ``dW`` into the weight's registered gradient target (:func:`set_grad_targets`)."""

    @staticmethod
    def forward(ctx, x, weight, residual):
        x2 = x.reshape(-1, x.shape[-1])
        shape = (*x.shape[:-1], weight.shape[0])
        if residual is None:
            y = torch.mm(x2, weight.t())
        else:
            y = torch.addmm(residual.reshape(-1, weight.shape[0]), x2, weight.t())
        ctx.save_for_backward(x2, weight)
        ctx.param, ctx.shape, ctx.has_res = weight, x.shape, residual is not None
        return y.view(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[0])
        dx = torch.mm(dy2, weight).view(ctx.shape) if ctx.needs_input_grad[0] else None
        dw = _dw(dy2, x2, ctx.param) if ctx.needs_input_grad[1] else None
        dres = dy if ctx.has_res and ctx.needs_input_grad[2] else None
        return dx, dw, dres


class _MultiLinear(torch.autograd.Function):
    """``[x·W_iᵀ]`` for several weights over ONE input: the backward's ``dX = Σ dY_i·W_i`` is one
    GEMM plus beta = 1 accumulating GEMMs into the same buffer (autograd would sum the per-output
    input gradients with separate add passes: two per Llama block for q / k / v, one for w1 / w3)."""

    @staticmethod
    def forward(ctx, x, *weights):
        x2 = x.reshape(-1, x.shape[-1])
        ctx.save_for_backward(x2, *weights)
        ctx.params = weights  # (the parameter objects themselves: their .grad / registered target)
        ctx.shape = x.shape
        return tuple(torch.mm(x2, w.t()).view(*x.shape[:-1], w.shape[0]) for w in weights)

    @staticmethod
    def backward(ctx, *dys):
        x2, *weights = ctx.saved_tensors
        dx = None
        if ctx.needs_input_grad[0]:
            for dy, w in zip(dys, weights):
                if dy is None:
                    continue
                d2 = dy.reshape(-1, w.shape[0])
                dx = torch.mm(d2, w) if dx is None else dx.addmm_(d2, w)
            if dx is not None:
                dx = dx.view(ctx.shape)
        dws = [_dw(dy.reshape(-1, w.shape[0]), x2, ctx.params[i]) if dy is not None and ctx.needs_input_grad[1 + i]
               else None for i, (dy, w) in enumerate(zip(dys, weights))]
        return (dx, *dws)


def multi_linear(x: torch.Tensor, *weights: torch.Tensor):
    """``x·W_iᵀ`` for each weight (bias-free), the input gradient accumulated in GEMMs (see
    :class:`_MultiLinear`); the own GEMM's path (``XDDP_OWN_GEMM=1``) keeps one :func:`linear` per
    weight. ``XDDP_MULTI_LINEAR=0``: plain per-weight linears (A/B switch)."""
    if os.environ.get("XDDP_MULTI_LINEAR", "1") == "0" or _autocast_on(x) or any(own_gemm_ok(x, w) for w in weights) \
            or not all(w.dtype == x.dtype and w.dim() == 2 for w in weights):
        return tuple(linear(x, w) for w in weights)
    return _MultiLinear.apply(x, *weights)
