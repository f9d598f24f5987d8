"""Post-local SGD (reference: ``ddp_comm_hooks/post_localSGD_hook.py:13-124``, Lin et al. 2018).

Global all-reduce for the first ``start_localSGD_iter`` steps, then all-reduce only within
``subgroup`` (e.g. the GPUs of one node / one xGMI island) — a model averager
(``PeriodicModelAverager``) re-synchronizes parameters globally every ``period`` steps.
"""
from __future__ import annotations

import torch

from ... import distributed as xdist
from .default_hooks import _allreduce_fut


class PostLocalSGDState:
    __slots__ = ["process_group", "subgroup", "start_localSGD_iter", "post_local_gradient_allreduce", "iter"]

    def __init__(self, process_group, subgroup, start_localSGD_iter: int, post_local_gradient_allreduce: bool = True):
        self.process_group = process_group
        self.subgroup = subgroup
        self.start_localSGD_iter = start_localSGD_iter
        self.post_local_gradient_allreduce = post_local_gradient_allreduce
        self.iter = 0

    def maybe_increase_iter(self, bucket):
        if bucket.is_last():
            self.iter += 1


def post_localSGD_hook(state: PostLocalSGDState, bucket) -> torch.futures.Future:
    buf = bucket.buffer()
    if state.iter < state.start_localSGD_iter:
        state.maybe_increase_iter(bucket)
        return _allreduce_fut(state.process_group, buf)
    if not state.post_local_gradient_allreduce:
        fut = torch.futures.Future()
        fut.set_result(buf)
        return fut
    return _allreduce_fut(state.subgroup, buf)


class PeriodicModelAverager:
    """Average parameters across ``process_group`` every ``period`` steps after ``warmup_steps``."""

    def __init__(self, period: int, warmup_steps: int = 0, process_group=None):
        if period < 1:
            raise ValueError("period must be a positive integer")
        self.period, self.warmup_steps, self.step = period, warmup_steps, 0
        self.process_group = process_group

    def average_parameters(self, params):
        if self.step >= self.warmup_steps and (self.step - self.warmup_steps) % self.period == 0:
            pg = self.process_group if self.process_group is not None else xdist.get_default_group()
            params = [p for p in params if p is not None]
            if params:
                flat = torch.cat([p.detach().reshape(-1).float() for p in params])
                pg.allreduce(flat, xdist.ReduceOp.AVG).wait()
                off = 0
                with torch.no_grad():
                    for p in params:
                        p.copy_(flat[off: off + p.numel()].view_as(p))
                        off += p.numel()
        self.step += 1
