"""SyncBatchNorm over xddp process groups (reference: ``torch/nn/modules/_functions.py:7-200``,
``SyncBatchNorm.convert_sync_batchnorm``).

Forward: per-rank (count, mean, M2) in fp32 → one all-gather of a [3, C] block per rank →
Chan-merged global mean/var (numerically safe, no sum-of-squares cancellation) → normalize
(+ running-stat EMA with the global unbiased variance). Backward: per-rank Σdy and
Σdy·(x-mean) → one all-reduce of a [C, 2] block → dx; dweight / dbias stay local (DDP averages
them with the other gradients), as in the reference.

GPU NHWC inputs (channels_last, C % 8 == 0) run on the fused BN kernels of
``csrc/kernels/batch_norm.hip``: ``bn_moments`` (one stats pass) → RCCL all-gather →
``bn_stats_from_partials`` (the ranks are the groups of its Chan merge; also the running-stat
update) → ``bn_apply``; backward ``bn_grad_partials`` (one reduce pass) → RCCL all-reduce →
``bn_backward_from_partials`` → ``bn_backward_elem``. Three activation passes in all, no fp32
copies of the activation. Other inputs (CPU, NCHW) use the eager fp32 path below.
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
        # [C, 2] = (sum dy, sum dy·(x - mean)): the same payload layout as the native path, so ranks
        # that take different paths (layout / alignment differs) still reduce matching channels
        sums = torch.stack([dyf.sum(dims), (dyf * xmu).sum(dims)], dim=1).contiguous()
        local_sums = sums.clone()
        ctx.pg.allreduce(sums).wait()
        sum_dy, sum_dy_xmu = sums[:, 0], sums[:, 1]
        g = weight.float() if weight is not None else torch.ones(C, device=x.device)
        dx = (dyf - (sum_dy / n).view(shape) - xmu * (invstd ** 2 * sum_dy_xmu / n).view(shape)) \
            * (g * invstd).view(shape)
        dw = (local_sums[:, 1] * invstd).to(weight.dtype) if weight is not None else None
        db = local_sums[:, 0].to(weight.dtype) if weight is not None else None
        return dx.to(x.dtype), dw, db, None, None, None, None, None


def _native_ok(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.shape[1] % 8 == 0 and x.numel() > 0
            and x.dtype in (torch.bfloat16, torch.float16, torch.float32)
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0)


class _SyncBNNative(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, eps, momentum, pg):
        from .._native import load

        C = load()
        local = C.bn_moments(x)  # [3, C]: count, mean, M2
        gathered = torch.empty((pg.size(),) + tuple(local.shape), device=x.device, dtype=torch.float32)
        pg.allgather_into_tensor(gathered, local).wait()
        # M = 0: the finalize sums the gathered per-rank counts on the device, so uneven shards (a
        # short last batch, uneven samplers) get exact statistics without a host sync
        mean, invstd, ss = C.bn_stats_from_partials(gathered, 0, weight, bias, running_mean, running_var, None,
                                                    momentum, False, eps)
        y, _ = C.bn_apply(x, ss, None, False, False, None)
        count = gathered[:, 0, :1].sum(0)  # [1]: global rows behind the statistics (device)
        ctx.save_for_backward(x, weight, mean, invstd, count)
        ctx.pg = pg
        return y

    @staticmethod
    def backward(ctx, dy):
        from .._native import load

        C = load()
        x, weight, mean, invstd, count = ctx.saved_tensors
        part = C.bn_grad_partials(dy, x, mean)  # [blocks, C, 2]: sum dy, sum dy·(x - mean)
        local = part.sum(0, keepdim=True)
        total = local.clone()
        work = ctx.pg.allreduce(total)
        dw = db = None
        need_w = weight is not None and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2])
        if need_w:  # local dweight / dbias, computed while the all-reduce is in flight
            _, dw, db = C.bn_backward_from_partials(local, x.numel() // x.shape[1], weight, mean, invstd, True, False)
        work.wait()
        # the finalize scales the sums by 1/M: hand it sums / global count with M = 1 (exact for
        # uneven shards, no host sync)
        coef, _, _ = C.bn_backward_from_partials(total / count, 1, weight, mean, invstd, False, False)
        dx = C.bn_backward_elem(dy.contiguous(memory_format=torch.channels_last), x, mean, coef)
        return dx, dw, db, None, None, None, None, None


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
        if _native_ok(x):
            return _SyncBNNative.apply(x, self.weight, self.bias, rm, rv, self.eps, mom, pg)
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
