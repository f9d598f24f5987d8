"""Fused BatchNorm2d (+ residual add + ReLU) on xddp's NHWC HIP kernels.

Drop-in for ``nn.BatchNorm2d``: same parameters, buffers and state_dict keys (it *is* a
``BatchNorm2d`` subclass, so DDP buffer sync, ``convert_sync_batchnorm`` and checkpoints
see the standard layout). ``forward(x, residual=None, relu=False)`` fuses the
bottleneck/basic-block epilogue ``relu(bn(x) + residual)`` into one pass forward and one
backward (SURVEY.md §2.6 K3–K6, K9). Inputs that the kernels do not cover (NCHW layout,
C % 8 != 0, CPU, eval-mode autograd) take the equivalent PyTorch path.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import load

__all__ = ["FusedBatchNorm2d", "batch_norm_act"]


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, residual, relu, dual):
        C = load()
        ctx.set_materialize_grads(False)
        # ReLU mask: with a residual the mask depends on it, so the forward stores it as bits
        # (1/16 of a bf16 activation); without one it is recomputed from x*scale+shift
        keep_mask = relu and residual is not None
        y, mean, invstd, ss, bits = C.bn_forward(x, weight, bias, running_mean, running_var, nbt, True, momentum,
                                                 cma, eps, residual, relu, keep_mask)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.save_for_backward(x, bits if keep_mask else None, weight, mean, invstd, ss)
        if dual:
            # two consumers (next block's conv and its residual) get separate autograd outputs over
            # the same memory, so their gradients reach backward() unsummed: the kernels add them
            # in registers instead of an autograd add kernel over the whole activation
            return y, y.view_as(y)
        return y

    @staticmethod
    def backward(ctx, dy, dy2=None):
        C = load()
        x, bits, weight, mean, invstd, ss = ctx.saved_tensors
        if dy is None:
            dy, dy2 = dy2, None
        if dy is None:
            return (None,) * 12
        need_dw = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        dx, dw, db, dres = C.bn_backward(dy, x, None, weight, mean, invstd, ss, ctx.relu,
                                         ctx.has_res and ctx.needs_input_grad[9], need_dw, dy2, bits)
        return (dx, dw if ctx.needs_input_grad[1] else None, db if ctx.needs_input_grad[2] else None,
                None, None, None, None, None, None, dres if ctx.has_res else None, None, None)


def _kernel_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.size(1) % 8 == 0 and x.numel() > 0
            and x.is_contiguous(memory_format=torch.channels_last)
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.data_ptr() % 16 == 0)


def batch_norm_act(x, running_mean, running_var, weight=None, bias=None, training=True, momentum=0.1, eps=1e-5,
                   num_batches_tracked=None, residual: Optional[torch.Tensor] = None, relu: bool = False,
                   dual_output: bool = False):
    """Functional fused BN(+add)(+ReLU). ``momentum=None`` means cumulative moving average.
    ``dual_output=True`` returns ``(y, y_alias)`` for an output with two consumers."""
    use_kernel = _kernel_ok(x) and (residual is None or (residual.shape == x.shape and residual.dtype == x.dtype and
                                                         residual.is_contiguous(memory_format=torch.channels_last)))
    if use_kernel and training:
        cma = momentum is None
        return _BNAct.apply(x, weight, bias, running_mean, running_var, num_batches_tracked,
                            0.0 if cma else float(momentum), cma, float(eps), residual, relu, dual_output)
    if use_kernel and not training and not (torch.is_grad_enabled() and (
            x.requires_grad or (weight is not None and weight.requires_grad))):
        C = load()
        y = C.bn_forward(x, weight, bias, running_mean, running_var, None, False, 0.0, False, float(eps),
                         residual, relu)[0]
        return (y, y) if dual_output else y
    # reference path
    if training and num_batches_tracked is not None:
        num_batches_tracked.add_(1)
        if momentum is None:
            momentum = 1.0 / float(num_batches_tracked)
    y = F.batch_norm(x, running_mean, running_var, weight, bias, training, momentum if momentum is not None else 0.0,
                     eps)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return (y, y) if dual_output else y


class FusedBatchNorm2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` with an NHWC HIP kernel and optional fused residual-add + ReLU."""

    supports_add_relu = True
    fuses_relu = True

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True, device=None,
                 dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device, dtype)
        self.relu = False

    def forward(self, x, residual: Optional[torch.Tensor] = None, relu: Optional[bool] = None,
                dual_output: bool = False):
        self._check_input_dim(x)
        relu = self.relu if relu is None else relu
        training = self.training or not self.track_running_stats
        rm = self.running_mean if (not self.training or self.track_running_stats) else None
        rv = self.running_var if (not self.training or self.track_running_stats) else None
        nbt = self.num_batches_tracked if (self.training and self.track_running_stats) else None
        return batch_norm_act(x, rm, rv, self.weight, self.bias, training, self.momentum, self.eps, nbt, residual,
                              relu, dual_output)

    def extra_repr(self):
        return super().extra_repr() + (", relu=True" if self.relu else "")
