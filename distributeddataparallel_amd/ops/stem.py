"""ResNet stem on own kernels: conv 7x7/s2 (3 -> 64) -> BatchNorm -> ReLU -> maxpool 3x3/s2.

Forward: ``stem_conv_forward`` (implicit GEMM from an LDS halo, BN statistics reduced in its
epilogue) -> ``bn_stats_from_partials`` -> ``stem_pool_forward`` (normalize + ReLU + pool in one
pass). Neither a separate statistics pass over the conv output nor the normalized activation
exists. Backward: ``stem_pool_bn_backward`` twice (BN partial sums, then dX, the pooled gradient
and the ReLU mask rebuilt on the fly) -> ``stem_conv_wgrad``. (r4/r5: forming the conv-output
gradient tile by tile inside the weight-gradient kernel instead needed more than 256 VGPRs and ran
one wave per SIMD, 555 us vs 176 + 130 us; removed.) The image needs no gradient, so there is no
input-gradient pass (if it does, torch's convolution backward adds it).
Kernels: csrc/kernels/stem_conv.hip, csrc/kernels/pool.hip.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["resnet_stem", "stem_supported"]


class _Stem(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, dual):
        C = load()
        ctx.set_materialize_grads(False)
        y, part = C.stem_conv_forward(x, w)
        M = y.numel() // y.shape[1]
        mean, invstd, ss = C.bn_stats_from_partials(part, M, weight, bias, running_mean, running_var, nbt, momentum,
                                                    cma, eps)
        if nbt is not None:
            nbt.add_(1)
        out, idx = C.stem_pool_forward(y, ss)
        ctx.save_for_backward(x, w, y, idx, weight, mean, invstd, ss)
        if dual:
            return out, out.view_as(out)
        return out

    @staticmethod
    def backward(ctx, dy, dy2=None):
        C = load()
        x, w, y, idx, weight, mean, invstd, ss = ctx.saved_tensors
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return (None,) * 11
        M = y.numel() // y.shape[1]
        need_bn = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        part = C.stem_pool_bn_backward(dy, dy2, idx, y, ss, mean)
        coef, dgamma, dbeta = C.bn_backward_from_partials(part, M, weight, mean, invstd, need_bn, False)
        dx = dw = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            dconv = C.stem_pool_bn_backward(dy, dy2, idx, y, ss, mean, coef)
            if ctx.needs_input_grad[1]:
                dw = C.stem_conv_wgrad(dconv, x, w)
            if ctx.needs_input_grad[0]:
                dx = torch.ops.aten.convolution_backward(dconv, x, w, None, [2, 2], [3, 3], [1, 1], False, [0, 0], 1,
                                                         [True, False, False])[0]
        return (dx, dw, dgamma if ctx.needs_input_grad[2] else None, dbeta if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, None, None)


def _single(v):
    return v[0] if isinstance(v, (tuple, list)) else v


def stem_supported(x, conv, bn, pool) -> bool:
    if os.environ.get("XDDP_STEM_CONV", "1") == "0":
        return False
    return (x.is_cuda and x.dim() == 4 and x.shape[1] == 3 and x.dtype == torch.bfloat16
            and x.is_contiguous(memory_format=torch.channels_last)
            and conv.weight.dtype == torch.bfloat16 and tuple(conv.weight.shape) == (64, 3, 7, 7)
            and conv.bias is None and _single(conv.stride) == 2 and _single(conv.padding) == 3
            and _single(conv.dilation) == 1 and conv.groups == 1
            and tuple(conv.stride) == (2, 2) and tuple(conv.padding) == (3, 3)
            and bn.training and bn.track_running_stats
            and (_single(pool.kernel_size), _single(pool.stride), _single(pool.padding)) == (3, 2, 1)
            and _single(pool.dilation) == 1 and not pool.ceil_mode)


def resnet_stem(x, conv, bn, pool, dual: bool = False):
    """``pool(relu(bn(conv(x))))`` on the own stem kernels (caller checks :func:`stem_supported`)."""
    cma = bn.momentum is None
    return _Stem.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked,
                       0.0 if cma else float(bn.momentum), cma, float(bn.eps), dual)


def _reference(x, w, weight, bias, eps=1e-5):  # fp32 math of the same op (tests)
    y = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    y = F.batch_norm(y, None, None, weight.float(), bias.float(), True, 0.0, eps)
    return F.max_pool2d(F.relu(y), 3, 2, 1)
