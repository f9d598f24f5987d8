"""SyncBatchNorm over xddp process groups (reference: ``torch/nn/modules/_functions.py:7-200``,
``SyncBatchNorm.convert_sync_batchnorm``).

Forward: per-rank (count, mean, M2) in fp32 → one all-gather of a [3, C] block per rank →
Chan-merged global mean/var (numerically safe, no sum-of-squares cancellation) → normalize
(+ running-stat EMA with the global unbiased variance). Backward: per-rank Σdy and
Σdy·(x-mean) → one all-reduce of a [2, C] block → dx. Works on both backends (CPU tensors on
``cpu``, GPU tensors on ``rccl``).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn

from .. import distributed as xdist


def _chan_merge(counts, means, m2s):
    n = counts.sum(0)
    mean = (counts * means).sum(0) / n.clamp_min(1)
    m2 = (m2s + counts * (means - mean) ** 2).sum(0)
    return n, mean, m2


class _SyncBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, pg):
        C = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        xf = x.float()
        cnt = torch.full((C,), float(xf.numel() // C), device=x.device)
        var, mean = torch.var_mean(xf, dim=dims, unbiased=False)
        m2 = var * cnt
        local = torch.stack([cnt, mean, m2])  # [3, C]
        world = pg.size()
        gathered = torch.empty((world, 3, C), device=x.device, dtype=torch.float32)
        pg.allgather_into_tensor(gathered, local.contiguous()).wait()
        n, gmean, gm2 = _chan_merge(gathered[:, 0], gathered[:, 1], gathered[:, 2])
        gvar = gm2 / n
        invstd = torch.rsqrt(gvar + eps)
        if running_mean is not None:
            with torch.no_grad():
                unbiased = gm2 / (n - 1).clamp_min(1)
                running_mean.mul_(1 - momentum).add_(gmean.to(running_mean.dtype), alpha=momentum)
                running_var.mul_(1 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
        shape = [1, C] + [1] * (x.dim() - 2)
        y = (xf - gmean.view(shape)) * invstd.view(shape)
        if weight is not None:
            y = y * weight.float().view(shape) + bias.float().view(shape)
        ctx.save_for_backward(x, weight, gmean, invstd, n)
        ctx.pg = pg
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, dy):
        x, weight, mean, invstd, n = ctx.saved_tensors
        C = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        shape = [1, C] + [1] * (x.dim() - 2)
        dyf, xf = dy.float(), x.float()
        xmu = xf - mean.view(shape)
        sums = torch.stack([dyf.sum(dims), (dyf * xmu).sum(dims)])
        local_sums = sums.clone()
        ctx.pg.allreduce(sums).wait()
        sum_dy, sum_dy_xmu = sums[0], sums[1]
        g = weight.float() if weight is not None else torch.ones(C, device=x.device)
        dx = (dyf - (sum_dy / n).view(shape) - xmu * (invstd ** 2 * sum_dy_xmu / n).view(shape)) \
            * (g * invstd).view(shape)
        dw = (local_sums[1] * invstd).to(weight.dtype) if weight is not None else None
        db = local_sums[0].to(weight.dtype) if weight is not None else None
        return dx.to(x.dtype), dw, db, None, None, None, None, None


class SyncBatchNorm(nn.modules.batchnorm._BatchNorm):
    def __init__(self, num_features, eps=1e-5, momentum: Optional[float] = 0.1, affine=True,
                 track_running_stats=True, process_group=None, device=None, dtype=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats, device, dtype)
        self.process_group = process_group

    def _check_input_dim(self, x):
        if x.dim() < 2:
            raise ValueError(f"expected at least 2D input (got {x.dim()}D input)")

    def forward(self, x):
        self._check_input_dim(x)
        mom = 0.0 if self.momentum is None else self.momentum
        if self.training and self.track_running_stats:
            self.num_batches_tracked.add_(1)
            if self.momentum is None:
                mom = 1.0 / float(self.num_batches_tracked)
        use_sync = self.training and xdist.is_initialized()
        if not use_sync:
            return nn.functional.batch_norm(
                x, self.running_mean if not self.training or self.track_running_stats else None,
                self.running_var if not self.training or self.track_running_stats else None,
                self.weight, self.bias, self.training or not self.track_running_stats, mom, self.eps)
        pg = self.process_group if self.process_group is not None else xdist.get_default_group()
        rm = self.running_mean if self.track_running_stats else None
        rv = self.running_var if self.track_running_stats else None
        return _SyncBN.apply(x, self.weight, self.bias, rm, rv, self.eps, mom, pg)

    @classmethod
    def convert_sync_batchnorm(cls, module: nn.Module, process_group=None) -> nn.Module:
        out = module
        if isinstance(module, nn.modules.batchnorm._BatchNorm):
            out = cls(module.num_features, module.eps, module.momentum, module.affine, module.track_running_stats,
                      process_group)
            if module.affine:
                with torch.no_grad():
                    out.weight = module.weight
                    out.bias = module.bias
            out.running_mean = module.running_mean
            out.running_var = module.running_var
            out.num_batches_tracked = module.num_batches_tracked
            out.training = module.training
        for name, child in module.named_children():
            out.add_module(name, cls.convert_sync_batchnorm(child, process_group))
        del module
        return out
