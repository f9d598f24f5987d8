"""Quantized all-gather comm hooks (reference: ``ddp_comm_hooks/quantization_hooks.py:46-220``).

Each rank quantizes its bucket to uint8 with its own affine (scale, zero-point) — per
tensor or per channel row block — all-gathers the uint8 payload plus the quantization
parameters, dequantizes every rank's contribution and averages locally.
"""
from __future__ import annotations

import torch

from ... import distributed as xdist


def _qparams(t: torch.Tensor):
    lo, hi = t.min(), t.max()
    scale = ((hi - lo) / 255.0).clamp_min(1e-12)
    zp = (-lo / scale).round().clamp(0, 255)
    return scale, zp


def _gather_then(pg, payloads, finish) -> torch.futures.Future:
    """All-gather each (out, in) pair without blocking the autograd thread; ``finish`` runs when
    both payloads have arrived (on GPU: once the caller's stream is ordered after them)."""
    futs = [pg.allgather_into_tensor(out, inp).get_future() for out, inp in payloads]
    return torch.futures.collect_all(futs).then(lambda _: finish())


def quantization_pertensor_hook(process_group, bucket) -> torch.futures.Future:
    pg = process_group if process_group is not None else xdist.get_default_group()
    w = pg.size()
    buf = bucket.buffer()
    x = buf.float()
    scale, zp = _qparams(x)
    q = (x / scale + zp).round().clamp(0, 255).to(torch.uint8)
    qp = torch.stack([scale, zp]).float()
    all_q = torch.empty(w * q.numel(), dtype=torch.uint8, device=q.device)
    all_p = torch.empty(w * 2, dtype=torch.float32, device=q.device)

    def finish():
        p = all_p.view(w, 2)
        deq = (all_q.view(w, -1).float() - p[:, 1:2]) * p[:, 0:1]
        buf.copy_(deq.mean(0).to(buf.dtype))
        return buf

    return _gather_then(pg, [(all_q, q), (all_p, qp)], finish)


def quantization_perchannel_hook(process_group, bucket, bucket_size: int = 512) -> torch.futures.Future:
    pg = process_group if process_group is not None else xdist.get_default_group()
    w = pg.size()
    buf = bucket.buffer()
    n = buf.numel()
    rows = (n + bucket_size - 1) // bucket_size
    x = torch.zeros(rows * bucket_size, dtype=torch.float32, device=buf.device)
    x[:n] = buf.float()
    x = x.view(rows, bucket_size)
    lo, hi = x.min(1, keepdim=True).values, x.max(1, keepdim=True).values
    scale = ((hi - lo) / 255.0).clamp_min(1e-12)
    zp = (-lo / scale).round().clamp(0, 255)
    q = (x / scale + zp).round().clamp(0, 255).to(torch.uint8)
    qp = torch.cat([scale, zp], 1).contiguous()
    all_q = torch.empty((w,) + tuple(q.shape), dtype=torch.uint8, device=buf.device)
    all_p = torch.empty((w,) + tuple(qp.shape), dtype=torch.float32, device=buf.device)

    def finish():
        deq = (all_q.float() - all_p[..., 1:2]) * all_p[..., 0:1]
        buf.copy_(deq.mean(0).reshape(-1)[:n].to(buf.dtype))
        return buf

    return _gather_then(pg, [(all_q, q), (all_p, qp)], finish)
