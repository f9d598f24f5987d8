"""NHWC max-pool with a one-byte in-window argmax (ResNet stem)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import load

__all__ = ["FusedMaxPool2d", "stem_bn_relu_maxpool", "global_avg_pool"]


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p, dual):
        ctx.set_materialize_grads(False)
        y, idx = load().maxpool_forward(x, k, s, p)
        ctx.save_for_backward(idx)
        ctx.meta = (x.shape, k, s, p)
        if dual:  # two consumers (block-0 conv1 and its downsample/residual): grads summed in-kernel
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, dy, dy2=None):
        (idx,) = ctx.saved_tensors
        shape, k, s, p = ctx.meta
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return None, None, None, None, None
        x_like = torch.empty(shape, device="meta")  # only the input shape is needed
        return load().maxpool_backward(dy, idx, x_like, k, s, p, dy2), None, None, None, None


class _StemBNPool(torch.autograd.Function):
    """bn (batch statistics) -> ReLU -> maxpool(3, 2, 1) with the normalized activation never
    materialized (csrc/kernels/pool.hip, stem_*): forward = one stats pass over y + one fused
    normalize/ReLU/pool pass; backward = partial-sums pass + dX pass, both rebuilding the pooled
    gradient and the ReLU mask on the fly."""

    @staticmethod
    def forward(ctx, y, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, dual):
        C = load()
        ctx.set_materialize_grads(False)
        M = y.numel() // y.shape[1]
        moments = C.bn_moments(y)  # [3, C]
        mean, invstd, ss = C.bn_stats_from_partials(moments.unsqueeze(0), M, weight, bias, running_mean, running_var,
                                                    nbt, momentum, cma, eps)
        if nbt is not None:
            nbt.add_(1)
        out, idx = C.stem_pool_forward(y, ss)
        ctx.save_for_backward(y, idx, weight, mean, invstd, ss)
        if dual:  # block-0 conv1 and its downsample: gradients summed in-kernel
            return out, out.view_as(out)
        return out

    @staticmethod
    def backward(ctx, dy, dy2=None):
        C = load()
        y, idx, weight, mean, invstd, ss = ctx.saved_tensors
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return (None,) * 10
        M = y.numel() // y.shape[1]
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        part = C.stem_pool_bn_backward(dy, dy2, idx, y, ss, mean)
        coef, dw, db = C.bn_backward_from_partials(part, M, weight, mean, invstd, need_w, False)
        dx = C.stem_pool_bn_backward(dy, dy2, idx, y, ss, mean, coef) if ctx.needs_input_grad[0] else None
        return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, None)


def stem_bn_relu_maxpool(y, bn, pool, dual: bool = False):
    """``pool(relu(bn(y)))`` for a training-mode FusedBatchNorm2d and a 3x3/s2/p1 max-pool on an
    NHWC tensor; returns ``None`` when the fused kernels do not cover the case (caller falls back)."""
    k, s, p = _single(pool.kernel_size), _single(pool.stride), _single(pool.padding)
    if not (bn.training and bn.track_running_stats and (k, s, p) == (3, 2, 1) and _single(pool.dilation) == 1
            and not pool.ceil_mode and y.is_cuda and y.dim() == 4 and y.size(1) % 8 == 0 and 256 % (y.size(1) // 8) == 0
            and y.is_contiguous(memory_format=torch.channels_last) and y.data_ptr() % 16 == 0
            and y.dtype in (torch.bfloat16, torch.float16, torch.float32)):
        return None
    cma = bn.momentum is None
    return _StemBNPool.apply(y, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                             0.0 if cma else float(bn.momentum), cma, float(bn.eps), dual)


def _single(v):
    return v[0] if isinstance(v, (tuple, list)) else v


class FusedMaxPool2d(nn.MaxPool2d):
    dual_output = False  # set by models whose pooled output feeds two consumers

    def forward(self, x):
        k, s, p = _single(self.kernel_size), _single(self.stride), _single(self.padding)
        ok = (x.is_cuda and x.dim() == 4 and x.size(1) % 8 == 0 and x.is_contiguous(memory_format=torch.channels_last)
              and _single(self.dilation) == 1 and not self.ceil_mode and not self.return_indices and k * k <= 255
              and all(isinstance(v, int) or len(set(v)) == 1 for v in (self.kernel_size, self.stride, self.padding)))
        if not ok:
            y = super().forward(x)
            return (y, y) if self.dual_output else y
        return _MaxPool.apply(x, k, s, p, self.dual_output)


class _GlobalAvgPool(torch.autograd.Function):
    """[B, C, H, W] channels_last -> [B, C] spatial mean. The backward writes the broadcast
    gradient g / HW straight into a channels_last tensor (one write pass). ``nn.AdaptiveAvgPool2d``
    backward produces an NCHW gradient that autograd then converts to channels_last with a strided
    transpose copy: 102 us per ResNet-50 bs256 step (rocprof), against ~15 us here."""

    @staticmethod
    def forward(ctx, x):
        ctx.shape, ctx.dtype = x.shape, x.dtype
        ctx.like = torch.empty((1,), dtype=x.dtype, device=x.device).expand(x.shape)  # shape/dtype carrier
        return x.mean((2, 3))

    @staticmethod
    def backward(ctx, g):
        B, C, H, W = ctx.shape
        if g.is_cuda and C % 8 == 0 and g.dtype in (torch.float32, torch.bfloat16):
            # one 16-B store per 8 channels of a pixel (pool.hip gap_bwd_kernel): 36 -> ~10 us at
            # the ResNet-50 bs256 shape vs the broadcast copy below
            return load().global_avg_pool_backward(g.contiguous(), ctx.like)
        out = torch.empty((B, C, H, W), dtype=ctx.dtype, device=g.device, memory_format=torch.channels_last)
        out.copy_((g / (H * W)).to(ctx.dtype)[:, :, None, None].expand(B, C, H, W))
        return out


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``flatten(AdaptiveAvgPool2d(1)(x), 1)`` with a channels_last backward."""
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) and torch.is_grad_enabled():
        return _GlobalAvgPool.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
