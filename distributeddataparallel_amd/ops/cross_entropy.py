"""Softmax cross-entropy on xddp's HIP kernels (``csrc/kernels/cross_entropy.hip``) for the
Llama-3-8B LM head of BASELINE.json config 5: bf16 logits [rows, vocab], fp32 math, mean over
the non-ignored rows — ``F.cross_entropy(logits.float(), target)`` without the 2.1 GB fp32 copy
of the logits, its zero-filled fp32 gradient and the casts (one read of the logits forward, one
read + one bf16 write backward). CPU tensors and other dtypes / shapes fall back to torch.

Targets outside ``[0, classes)`` other than ``ignore_index`` are an error, as in torch. The
kernel makes that row's loss NaN (so the step's loss shows it at once), gives it no gradient and
sets a per-device flag; the flag is copied to pinned host memory behind the kernel and read at
the next call (or by :func:`check_targets`), which raises ``IndexError`` — no host sync per step.
``XDDP_XENT_CHECK=sync`` checks right after the forward instead (a sync per call).

Under HIP-graph capture (``bench.py --graphs``, ``utils/graphs.py``) the host-side check, the flag
copy and the event are skipped: an event query or record inside a capture is not allowed, and a
replay could not run the host check anyway. The device flag is still set and the row's loss is
still NaN, so a bad target shows in the replayed loss; the next eager call raises as usual.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._native import load

__all__ = ["cross_entropy", "check_targets"]

_FLAGS: dict = {}  # device index -> (device flag int32[1], pinned host copy, event of the copy)


def _flag(dev: torch.device):
    f = _FLAGS.get(dev.index)
    if f is None:
        f = (torch.zeros(1, dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int32).pin_memory(),
             torch.cuda.Event())
        _FLAGS[dev.index] = f
    return f


def check_targets(block: bool = False) -> None:
    """Raise ``IndexError`` if a fused cross-entropy call so far saw a target outside
    ``[0, classes)`` (other than ``ignore_index``). Without ``block`` only copies that already
    landed are looked at (no sync)."""
    for dev, (flag, host, ev) in _FLAGS.items():
        if block:
            ev.synchronize()
        elif not ev.query():
            continue
        if int(host[0]) != 0:
            flag.zero_()
            host.zero_()
            raise IndexError(f"cross_entropy: a target is out of bounds (not in [0, classes) and not "
                             f"ignore_index) on cuda:{dev}")


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index):
        C = load()
        capturing = torch.cuda.is_current_stream_capturing()
        if not capturing:
            check_targets()  # an earlier call's invalid target surfaces here, without a sync
        flag, host, ev = _flag(logits.device)
        loss_rows, lse = C.cross_entropy_forward(logits, target, ignore_index, flag)
        if not capturing:
            host.copy_(flag, non_blocking=True)
            ev.record(torch.cuda.current_stream(logits.device))
            if os.environ.get("XDDP_XENT_CHECK") == "sync":
                check_targets(block=True)
        count = (target != ignore_index).sum().clamp_min(1).to(torch.float32)
        ctx.save_for_backward(logits, target, lse, count)
        ctx.ignore_index = ignore_index
        return loss_rows.sum() / count

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, count = ctx.saved_tensors
        gscale = (g.to(torch.float32) / count).reshape(1).contiguous()
        d = load().cross_entropy_backward(logits, target, lse, gscale, ctx.ignore_index)
        return d, None, None


def cross_entropy(logits: torch.Tensor, target: torch.Tensor, ignore_index: int = -100) -> torch.Tensor:
    """Mean softmax cross-entropy of ``logits`` [rows, classes] against ``target`` [rows]; bf16
    CUDA logits with a class count divisible by 8 run the fused kernels, anything else
    ``F.cross_entropy`` on the fp32 upcast."""
    if (logits.is_cuda and logits.dtype == torch.bfloat16 and logits.dim() == 2 and logits.size(1) % 8 == 0
            and target.dtype == torch.long and target.dim() == 1):
        return _CrossEntropy.apply(logits.contiguous(), target.contiguous(), ignore_index)
    return F.cross_entropy(logits.float(), target, ignore_index=ignore_index)
