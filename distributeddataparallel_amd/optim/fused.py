"""Fused multi-tensor optimizers and grad-norm clipping on HIP kernels.

Reference hot path: ``optim.SGD`` → one ``_foreach_add_`` over all
params. Here one native launch per (dtype-group × 40 tensors) does the full update —
weight decay, momentum/Nesterov, Adam moments, bias correction, and optionally fp32
master weights for bf16/fp16 models — reading each operand once with 16-byte loads.
``grad_scale`` (a device scalar) lets a clip coefficient or loss-scale be applied inside
the same pass without a host sync.

CPU tensors take an equivalent torch reference path (the GPU-free test backend).
"""
from __future__ import annotations

from collections import defaultdict
from typing import Iterable, List, Optional

import torch
from torch.optim import Optimizer

from .._native import load

__all__ = ["FusedSGD", "FusedAdamW", "FusedAdam", "clip_grad_norm_", "grad_norm"]


def _group_key(p: torch.Tensor, g: torch.Tensor):
    return (p.device, p.dtype, g.dtype)


def _dense_like(p: torch.Tensor) -> torch.Tensor:
    return torch.empty_strided(p.size(), p.stride(), dtype=torch.float32, device=p.device)


def _flat_range(t: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
    """Elements [lo, hi) of a dense (possibly permuted-stride) tensor in memory order, as a 1-D view."""
    expect = 1
    for st, sz in sorted((st, sz) for st, sz in zip(t.stride(), t.size()) if sz != 1):
        if st != expect:
            raise ValueError("slice updates need dense parameters / gradients / states")
        expect *= sz
    return t.as_strided((hi - lo,), (1,), t.storage_offset() + lo)


class FusedSGD(Optimizer):
    """SGD with momentum/dampening/Nesterov/weight decay (torch.optim.SGD semantics).

    ``master_weights=True`` keeps fp32 master copies for low-precision params.
    """

    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, maximize: bool = False,
                 master_weights: bool = False):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                        nesterov=nesterov, maximize=maximize, master_weights=master_weights)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[torch.Tensor] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        C = load()
        for group in self.param_groups:
            buckets = defaultdict(lambda: ([], [], [], []))
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                first = "momentum_buffer" not in st
                if group["momentum"] != 0 and first:
                    st["momentum_buffer"] = _dense_like(p)
                use_master = group["master_weights"] and p.dtype in (torch.bfloat16, torch.float16)
                if use_master and "master" not in st:
                    st["master"] = p.detach().float().clone(memory_format=torch.preserve_format)
                key = _group_key(p, p.grad) + (first, use_master)
                b = buckets[key]
                b[0].append(st["master"] if use_master else p)
                b[1].append(p.grad)
                b[2].append(st.get("momentum_buffer"))
                b[3].append(p)
            for (dev, pdt, gdt, first, use_master), (ps, gs, bufs, orig) in buckets.items():
                mom = group["momentum"]
                bufs = bufs if mom != 0 else []
                if dev.type == "cuda" and use_master:  # one pass: update fp32 masters, round into the params
                    C.fused_sgd_master(ps, gs, bufs, orig, group["lr"], mom, group["dampening"],
                                       group["weight_decay"], group["nesterov"], group["maximize"], first, grad_scale)
                elif dev.type == "cuda":
                    C.fused_sgd(ps, gs, bufs, group["lr"], mom, group["dampening"], group["weight_decay"],
                                group["nesterov"], group["maximize"], first, grad_scale)
                else:
                    self._cpu_step(ps, gs, bufs, group, first, grad_scale)
                    if use_master:
                        for m, p in zip(ps, orig):
                            p.copy_(m)
        return loss

    @staticmethod
    def _cpu_step(ps, gs, bufs, group, first, grad_scale):
        lr, mom, damp, wd = group["lr"], group["momentum"], group["dampening"], group["weight_decay"]
        for i, (p, g) in enumerate(zip(ps, gs)):
            d = g.float()
            if grad_scale is not None:
                d = d * grad_scale.float()
            if group["maximize"]:
                d = -d
            if wd != 0:
                d = d + wd * p.float()
            if mom != 0:
                buf = bufs[i]
                if first:
                    buf.copy_(d)
                else:
                    buf.mul_(mom).add_(d, alpha=1 - damp)
                d = d + mom * buf if group["nesterov"] else buf
            p.copy_(p.float() - lr * d)


class FusedAdamW(Optimizer):
    """Adam / AdamW (decoupled weight decay) with fp32 moments (torch.optim semantics, no amsgrad)."""

    _decoupled = True

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 maximize: bool = False, master_weights: bool = False, amsgrad: bool = False):
        if amsgrad:
            raise NotImplementedError("amsgrad is not supported by the fused kernel")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, maximize=maximize,
                        master_weights=master_weights)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: Optional[torch.Tensor] = None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        C = load()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            buckets = defaultdict(lambda: ([], [], [], [], [], []))
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if "step" not in st:
                    st["step"] = 0
                    st["exp_avg"] = _dense_like(p).zero_()
                    st["exp_avg_sq"] = _dense_like(p).zero_()
                    if group["master_weights"] and p.dtype in (torch.bfloat16, torch.float16):
                        st["master"] = p.detach().float().clone(memory_format=torch.preserve_format)
                st["step"] += 1
                key = _group_key(p, p.grad) + (st["step"], "master" in st)
                b = buckets[key]
                b[0].append(p)
                b[1].append(p.grad)
                b[2].append(st["exp_avg"])
                b[3].append(st["exp_avg_sq"])
                if "master" in st:
                    b[4].append(st["master"])
            for (dev, pdt, gdt, step, has_master), (ps, gs, m1, m2, masters, _) in buckets.items():
                if dev.type == "cuda":
                    C.fused_adam(ps, gs, m1, m2, masters, group["lr"], b1, b2, group["eps"], group["weight_decay"],
                                 step, self._decoupled, group["maximize"], grad_scale)
                else:
                    self._cpu_step(ps, gs, m1, m2, masters, group, step, grad_scale)
        return loss

    def _group_index(self, p):
        if not hasattr(self, "_group_of"):
            self._group_of = {id(q): gi for gi, grp in enumerate(self.param_groups) for q in grp["params"]}
        return self._group_of.get(id(p))

    def _init_state(self, p, group):
        st = self.state[p]
        if "step" not in st:
            st["step"] = 0
            st["exp_avg"] = _dense_like(p).zero_()
            st["exp_avg_sq"] = _dense_like(p).zero_()
            if group["master_weights"] and p.dtype in (torch.bfloat16, torch.float16):
                st["master"] = p.detach().float().clone(memory_format=torch.preserve_format)
        return st

    @torch.no_grad()
    def step_params(self, params, grads):
        """Step only ``params`` with the given gradients (e.g. one DDP bucket's reduced views, from
        an overlapped-optimizer comm hook): same update as ``step`` for those parameters."""
        live = [(p, g) for p, g in zip(params, grads) if g is not None and self._group_index(p) is not None]
        self.advance([p for p, _ in live])
        self.step_slices([(p, g, 0, p.numel()) for p, g in live])

    @torch.no_grad()
    def advance(self, params):
        """Start this step for ``params`` (state created on first use, step count + 1) without
        updating them; :meth:`step_slices` then updates them piecewise with that step count."""
        for p in params:
            gi = self._group_index(p)
            if gi is not None:
                self._init_state(p, self.param_groups[gi])["step"] += 1

    @torch.no_grad()
    def step_slices(self, pieces):
        """Update element ranges of parameters: ``pieces`` = ``[(param, grad, lo, hi)]`` with
        ``[lo, hi)`` in memory order of the (dense) param; ``grad`` has the param's shape and
        strides. Uses each param's current step count (:meth:`advance` first). AdamW is elementwise,
        so updating a param in several slices is bitwise the same as updating it at once — the
        overlapped optimizer steps a chunked tail bucket this way, chunk by chunk as each chunk's
        all-reduce lands."""
        C = load()
        per_group = defaultdict(list)
        for p, g, lo, hi in pieces:
            gi = self._group_index(p)
            if gi is not None and g is not None and hi > lo:
                per_group[gi].append((p, g, lo, hi))
        for gi, items in per_group.items():
            group = self.param_groups[gi]
            b1, b2 = group["betas"]
            buckets = defaultdict(lambda: ([], [], [], [], [], []))
            for p, g, lo, hi in items:
                st = self._init_state(p, group)
                if st["step"] == 0:
                    raise RuntimeError("step_slices before advance() for this step")
                b = buckets[_group_key(p, g) + (st["step"], "master" in st)]
                whole = lo == 0 and hi == p.numel()
                cut = (lambda t: t) if whole else (lambda t: _flat_range(t, lo, hi))
                b[0].append(cut(p))
                b[1].append(cut(g))
                b[2].append(cut(st["exp_avg"]))
                b[3].append(cut(st["exp_avg_sq"]))
                if "master" in st:
                    b[4].append(cut(st["master"]))
            for (dev, pdt, gdt, step, has_master), (ps, gs, m1, m2, masters, _) in buckets.items():
                if dev.type == "cuda":
                    C.fused_adam(ps, gs, m1, m2, masters, group["lr"], b1, b2, group["eps"], group["weight_decay"],
                                 step, self._decoupled, group["maximize"], None)
                else:
                    self._cpu_step(ps, gs, m1, m2, masters, group, step, None)

    def _cpu_step(self, ps, gs, m1, m2, masters, group, step, grad_scale):
        b1, b2 = group["betas"]
        lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
        bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
        for i, (p, g) in enumerate(zip(ps, gs)):
            w = masters[i] if masters else p.float()
            gg = g.float() * (grad_scale.float() if grad_scale is not None else 1.0)
            if group["maximize"]:
                gg = -gg
            if wd != 0:
                if self._decoupled:
                    w = w * (1 - lr * wd)
                else:
                    gg = gg + wd * w
            m1[i].mul_(b1).add_(gg, alpha=1 - b1)
            m2[i].mul_(b2).addcmul_(gg, gg, value=1 - b2)
            denom = (m2[i].sqrt() / (bc2 ** 0.5)).add_(eps)
            w = w - (lr / bc1) * m1[i] / denom
            if masters:
                masters[i].copy_(w)
            p.copy_(w)


class FusedAdam(FusedAdamW):
    """Adam with L2 (coupled) weight decay."""

    _decoupled = False

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, maximize=False,
                 master_weights=False, amsgrad=False):
        super().__init__(params, lr, betas, eps, weight_decay, maximize, master_weights, amsgrad)


def grad_norm(parameters: Iterable[torch.Tensor], max_norm: float = 0.0) -> torch.Tensor:
    """Total L2 norm of the grads (device scalar pair [norm, clip_coef]); no host sync on GPU."""
    grads = [p.grad for p in parameters if p.grad is not None]
    if not grads:
        return torch.tensor([0.0, 1.0])
    dev = grads[0].device
    if dev.type == "cuda":
        C = load()
        out = torch.empty(2, dtype=torch.float32, device=dev)
        by_dtype = defaultdict(list)
        for g in grads:
            by_dtype[g.dtype].append(g)
        if len(by_dtype) == 1:
            C.mt_l2norm(grads, out, float(max_norm))
            return out
        sq = torch.zeros(1, dtype=torch.float32, device=dev)
        for lst in by_dtype.values():
            C.mt_l2norm(lst, out, 0.0)
            sq += out[0] ** 2
        norm = sq.sqrt()
        coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(norm)
        return torch.cat([norm, coef])
    norm = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(g.float()) for g in grads]))
    coef = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(norm)
    return torch.stack([norm, coef])


def clip_grad_norm_(parameters: Iterable[torch.Tensor], max_norm: float, fused_into_optimizer: bool = False):
    """Clip grads by total L2 norm (torch.nn.utils.clip_grad_norm_ semantics).

    Returns the total norm (device tensor). With ``fused_into_optimizer=True`` the grads are
    not touched; instead ``(norm, coef)`` is returned so ``optimizer.step(grad_scale=coef)``
    applies the clip inside the fused update (one pass less over the gradients).
    """
    params = [p for p in parameters if p.grad is not None]
    nc = grad_norm(params, max_norm)
    if fused_into_optimizer:
        return nc[0], nc[1:2]
    grads = [p.grad for p in params]
    if grads and grads[0].device.type == "cuda":
        C = load()
        by_dtype = defaultdict(list)
        for g in grads:
            by_dtype[g.dtype].append(g)
        for lst in by_dtype.values():
            C.mt_scale_copy(lst, lst, 1.0, nc[1:2].contiguous())
    else:
        for g in grads:
            g.mul_(nc[1].to(g.dtype))
    return nc[0]
