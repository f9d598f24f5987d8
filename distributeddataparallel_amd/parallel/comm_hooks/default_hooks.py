"""Default DDP comm hooks (reference: ``torch/distributed/algorithms/ddp_comm_hooks/default_hooks.py:18-211``).

A hook is ``hook(state, bucket) -> torch.futures.Future[Tensor]``; ``state`` is a process group
(or None for the default group) and ``bucket`` a native ``GradBucket`` whose ``buffer()`` is
the flat gradient buffer of one bucket.
"""
from __future__ import annotations

from typing import Any, Callable

import torch

from ... import distributed as xdist


def _pg(process_group):
    return process_group if process_group is not None else xdist.get_default_group()


def _allreduce_fut(process_group, tensor: torch.Tensor) -> torch.futures.Future:
    pg = _pg(process_group)
    tensor.div_(pg.size())
    return pg.allreduce(tensor, xdist.ReduceOp.SUM).get_future().then(lambda fut: fut.value()[0])


def allreduce_hook(process_group, bucket) -> torch.futures.Future:
    """Divide by world size, then SUM all-reduce (what the native default does with ncclAvg)."""
    return _allreduce_fut(process_group, bucket.buffer())


def _compress_hook(dtype, process_group, bucket) -> torch.futures.Future:
    pg = _pg(process_group)
    buffer = bucket.buffer()
    compressed = buffer.to(dtype).div_(pg.size())

    def decompress(fut):
        buffer.copy_(fut.value()[0])
        return buffer

    return pg.allreduce(compressed, xdist.ReduceOp.SUM).get_future().then(decompress)


def fp16_compress_hook(process_group, bucket) -> torch.futures.Future:
    """Cast the bucket to fp16, all-reduce, cast back."""
    return _compress_hook(torch.float16, process_group, bucket)


def bf16_compress_hook(process_group, bucket) -> torch.futures.Future:
    """Cast the bucket to bf16, all-reduce, cast back."""
    return _compress_hook(torch.bfloat16, process_group, bucket)


class _CastBucket:
    """Present a cast copy of a bucket to a wrapped hook."""

    def __init__(self, bucket, buf):
        self._b = bucket
        self._buf = buf

    def buffer(self):
        return self._buf

    def __getattr__(self, name):
        return getattr(self._b, name)


def _compress_wrapper(dtype, hook: Callable[[Any, Any], torch.futures.Future]):
    def wrapped(hook_state, bucket) -> torch.futures.Future:
        buffer = bucket.buffer()
        cast = buffer.to(dtype)
        fut = hook(hook_state, _CastBucket(bucket, cast))

        def decompress(f):
            buffer.copy_(f.value() if isinstance(f.value(), torch.Tensor) else f.value()[0])
            return buffer

        return fut.then(decompress)

    return wrapped


def fp16_compress_wrapper(hook):
    return _compress_wrapper(torch.float16, hook)


def bf16_compress_wrapper(hook):
    return _compress_wrapper(torch.bfloat16, hook)
