"""Cross-rank replica check: are the model replicas still bit-identical?

DDP's contract (``ref:dpp.py:39``) is that every rank holds the same
parameters after every optimizer step: the all-reduced gradients are identical, so are the
updates. A transport or ordering bug in the collectives (a peer-memory kernel reading a stale
slot, buckets reduced in different orders on two ranks) breaks that silently: each rank's loss
still falls and the throughput still looks right. This module makes such a run fail loudly.

:func:`checksum` reduces a list of tensors (any dtypes) to three float64 numbers in ONE native
pass (``csrc/kernels/multi_tensor.hip`` ``mt_checksum``): the fp64 sum of the values and a 64-bit
XOR of position-mixed hashes of every element's raw bits (split into two exact 32-bit halves).
Per-block partials merge in a fixed order, so bit-equal tensors give bit-equal checksums.
:func:`check_replicas` all-gathers every rank's checksum, names the ranks that disagree with the
majority (ties: with rank 0), and optionally measures the largest absolute element difference
against rank 0's copy (one broadcast per dtype chunk, outside any timed region).

Users: ``bench.py`` after its timed region (``replicas_identical`` in the JSON line, non-zero exit
on divergence) and ``DistributedDataParallel`` every ``XDDP_CHECK_REPLICAS=N`` forwards (raises,
naming the ranks). Fault injection for the tests: ``XDDP_FAULT_CORRUPT="rank=R,iter=I"`` perturbs
one bucket after its all-reduce inside the Reducer (``csrc/reducer/reducer.cpp``).
"""
from __future__ import annotations

from collections import Counter
from typing import Dict, List, Sequence

import numpy as np
import torch

__all__ = ["checksum", "check_replicas"]

_M1, _M2 = np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _checksum_cpu(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """The same quantities on the host (CPU tensors; the hash is not comparable to the device one)."""
    total = 0.0
    h = np.uint64(0)
    with np.errstate(over="ignore"):
        for i, t in enumerate(tensors):
            t = t.detach().contiguous()
            if t.numel() == 0:
                continue
            if t.dtype.is_floating_point or t.dtype in (torch.int64, torch.int32, torch.int16, torch.int8,
                                                        torch.uint8):
                total += float(t.double().sum())
            raw = t.view(torch.uint8).numpy().reshape(t.numel(), t.element_size())
            bits = np.zeros(t.numel(), dtype=np.uint64)
            for b in range(t.element_size()):  # little-endian element bits
                bits |= raw[:, b].astype(np.uint64) << np.uint64(8 * b)
            seed = _mix64(np.array([i + 1], dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15))[0]
            pos = _mix64(seed + np.arange(t.numel(), dtype=np.uint64))
            h ^= np.bitwise_xor.reduce(_mix64(bits ^ pos))
    hv = int(h)
    return torch.tensor([total, float(hv & 0xFFFFFFFF), float(hv >> 32)], dtype=torch.float64)


def checksum(tensors: Sequence[torch.Tensor]) -> torch.Tensor:
    """float64 [3] = (sum of the values, hash low 32 bits, hash high 32 bits) over ``tensors``, on
    their device. Device tensors go through one native multi-tensor pass."""
    ts = [t.detach() for t in tensors if t.numel() > 0]
    if not ts:
        return torch.zeros(3, dtype=torch.float64)
    if ts[0].is_cuda:
        from .._native import load

        return load().mt_checksum([t if t.is_contiguous() else t.contiguous() for t in ts])
    return _checksum_cpu(ts)


def _max_abs_diff(tensors: List[torch.Tensor], pg, chunk_elems: int = 1 << 26) -> float:
    """max |t - t_rank0| over every floating tensor, MAX over ranks (rank 0's copies broadcast in
    per-dtype chunks of <= chunk_elems elements)."""
    worst = 0.0
    by_dtype: Dict[torch.dtype, List[torch.Tensor]] = {}
    for t in tensors:
        if t.dtype.is_floating_point and t.numel() > 0:
            by_dtype.setdefault(t.dtype, []).append(t.detach().reshape(-1))
    for ts in by_dtype.values():
        i = 0
        while i < len(ts):
            group, n = [], 0
            while i < len(ts) and (not group or n + ts[i].numel() <= chunk_elems):
                group.append(ts[i])
                n += ts[i].numel()
                i += 1
            flat = torch.cat(group)
            ref = flat.clone()
            pg.broadcast(ref, 0).wait()
            d = (flat.double() - ref.double()).abs().max()
            worst = max(worst, float(d))
    m = torch.tensor([worst], dtype=torch.float64, device=tensors[0].device)
    from ..distributed import ReduceOp

    pg.allreduce(m, ReduceOp.MAX).wait()
    return float(m.item())


def check_replicas(tensors: Sequence[torch.Tensor], pg, max_diff: bool = True) -> dict:
    """Compare ``tensors`` (the same list, in the same order, on every rank) across the ranks of
    ``pg``. Returns ``{"replicas_identical", "mismatch_ranks", "max_abs_diff", "checksum"}``;
    ``max_abs_diff`` is None unless ``max_diff``. Collective: every rank must call it."""
    tensors = [t for t in tensors if t is not None]
    cs = checksum(tensors)
    dev = tensors[0].device if tensors else torch.device("cpu")
    W = pg.size()
    mine = cs.to(dev)
    allv = torch.zeros(W * 3, dtype=torch.float64, device=dev)
    pg.allgather_into_tensor(allv, mine).wait()
    rows = [tuple(r) for r in allv.view(W, 3).cpu().tolist()]
    counts = Counter(rows)
    top = max(counts.values())
    majority = rows[0] if counts[rows[0]] == top else next(r for r in rows if counts[r] == top)
    bad = [r for r, v in enumerate(rows) if v != majority]
    out = {
        "replicas_identical": not bad,
        "mismatch_ranks": bad,
        "max_abs_diff": None,
        "checksum": {"sum": rows[pg.rank()][0], "hash": int(rows[pg.rank()][1]) | (int(rows[pg.rank()][2]) << 32)},
    }
    if max_diff and W > 1:
        out["max_abs_diff"] = _max_abs_diff(list(tensors), pg)
    return out
