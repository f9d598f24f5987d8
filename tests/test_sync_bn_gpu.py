"""SyncBatchNorm on the native NHWC BN kernels (bn_moments / bn_stats_from_partials / bn_apply,
bn_grad_partials / bn_backward_from_partials / bn_backward_elem): two ranks on one GPU (the cpu
backend stages the [3, C] / [C, 2] blocks through host memory), each holding half of a bf16
channels_last batch, against an fp32 torch BatchNorm2d over the whole batch."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from _dist_utils import run_ranks  # noqa: E402

pytestmark = pytest.mark.gpu


def _w_syncbn(rank, world, bounds=(0, 4, 8), eager_ranks=()):
    import torch.nn as nn

    from distributeddataparallel_amd.parallel.sync_batchnorm import SyncBatchNorm, _SyncBNNative

    torch.cuda.set_device(0)
    g = torch.Generator(device="cuda").manual_seed(7)
    N, C, H, W = 8, 64, 14, 14
    full = (torch.randn(N, C, H, W, device="cuda", generator=g) * 3 + 5).to(torch.bfloat16)
    dy_full = torch.randn(N, C, H, W, device="cuda", generator=g).to(torch.bfloat16)
    weight = torch.rand(C, device="cuda", generator=g) + 0.5
    bias = torch.randn(C, device="cuda", generator=g)

    ref = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        ref.weight.copy_(weight)
        ref.bias.copy_(bias)
    xr = full.float().requires_grad_(True)
    yr = ref(xr)
    yr.backward(dy_full.float())

    sbn = SyncBatchNorm(C).cuda()
    with torch.no_grad():
        sbn.weight.copy_(weight)
        sbn.bias.copy_(bias)
    sl = slice(bounds[rank], bounds[rank + 1])
    eager = rank in eager_ranks  # NCHW input: this rank takes the eager path, the others the native one
    fmt = torch.contiguous_format if eager else torch.channels_last
    x = full[sl].contiguous(memory_format=fmt).requires_grad_(True)
    calls = []
    orig = _SyncBNNative.forward

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    _SyncBNNative.forward = staticmethod(spy)
    try:
        y = sbn(x)
    finally:
        _SyncBNNative.forward = staticmethod(orig)
    assert bool(calls) != eager, "wrong SyncBatchNorm path"
    y.backward(dy_full[sl].contiguous(memory_format=fmt))

    def close(a, b, tol):
        err = ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()
        assert err < tol, err

    close(y, yr[sl], 1e-2)
    close(x.grad, xr.grad[sl], 2e-2)
    close(sbn.running_mean, ref.running_mean, 1e-4)
    close(sbn.running_var, ref.running_var, 1e-3)
    # dweight / dbias are local: their sum over ranks is the full-batch gradient
    from distributeddataparallel_amd import distributed as dist

    gw = torch.stack([sbn.weight.grad, sbn.bias.grad]).float().cpu()
    dist.all_reduce(gw)
    close(gw[0], ref.weight.grad.cpu(), 1e-2)
    close(gw[1], ref.bias.grad.cpu(), 1e-2)


def test_sync_batchnorm_native_two_ranks():
    run_ranks(_w_syncbn, world=2, backend="cpu")


def test_sync_batchnorm_native_uneven_shards():
    """5 + 3 rows: the statistics and the 1/M backward terms use the exact global count."""
    run_ranks(_w_syncbn, world=2, backend="cpu", args=((0, 5, 8),))


def test_sync_batchnorm_mixed_native_and_eager_ranks():
    """Rank 1's input is NCHW (eager path) while rank 0 runs the native kernels: the all-gathered
    [3, C] blocks and the all-reduced [C, 2] sums have the same layout on both paths."""
    run_ranks(_w_syncbn, world=2, backend="cpu", args=((0, 3, 8), (1,)))
