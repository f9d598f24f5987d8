"""NHWC max-pool with a one-byte in-window argmax (ResNet stem)."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .._native import load

__all__ = ["FusedMaxPool2d"]


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
