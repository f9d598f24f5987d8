"""Run the optimizer step for a bucket's parameters right after its all-reduce
(reference: ``ddp_comm_hooks/optimizer_overlap_hooks.py:17-163``, DDP ``_register_fused_optim``).

The step for bucket k overlaps the backward of the layers whose buckets are still
pending, instead of running after the whole backward.
"""
from __future__ import annotations

from typing import Any, Callable

import torch


class _OptimizerHookState:
    __slots__ = ["functional_optimizer", "params_to_optimize"]

    def __init__(self, optim_cls, params, *args, **kwargs):
        params = list(params)
        self.params_to_optimize = {id(p) for p in params}
        self.functional_optimizer = optim_cls(params, *args, **kwargs)


def _hook_then_optimizer(hook: Callable[[Any, Any], torch.futures.Future], optimizer_state: _OptimizerHookState):
    def hook_then_optimizer(hook_state, bucket) -> torch.futures.Future:
        fut = hook(hook_state, bucket)

        def apply_optim(f):
            grads = bucket.gradients()
            params = bucket.parameters()
            opt = optimizer_state.functional_optimizer
            chosen = [(p, g) for p, g in zip(params, grads) if id(p) in optimizer_state.params_to_optimize]
            saved = [(p, p.grad) for p, _ in chosen]
            for p, g in chosen:
                p.grad = g
            only = {id(p) for p, _ in chosen}
            groups = opt.param_groups
            stash = [g["params"] for g in groups]
            for g in groups:
                g["params"] = [p for p in g["params"] if id(p) in only]
            opt.step()
            for g, ps in zip(groups, stash):
                g["params"] = ps
            for p, old in saved:
                p.grad = old
            return bucket.buffer()

        return fut.then(apply_optim)

    return hook_then_optimizer
