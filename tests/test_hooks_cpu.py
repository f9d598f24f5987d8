"""Compression / local-SGD / optimizer-overlap hooks and SyncBatchNorm on the CPU backend (W=2)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from _dist_utils import run_ranks


def _mlp():
    from distributeddataparallel_amd.models import MLP

    torch.manual_seed(0)
    return MLP(784, 64, 10)


def _data(world, rank, n=3, seed=1):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        x = torch.randn(8 * world, 784, generator=g)
        y = torch.randint(0, 10, (8 * world,), generator=g)
        out.append((x, y, x[rank * 8:(rank + 1) * 8], y[rank * 8:(rank + 1) * 8]))
    return out


def _w_powersgd(rank, world, batched):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.parallel.comm_hooks.powerSGD_hook import (PowerSGDState,
                                                                                 batched_powerSGD_hook,
                                                                                 powerSGD_hook)

    m = _mlp()
    ddp = xddp.DDP(m)
    st = PowerSGDState(None, matrix_approximation_rank=4, start_powerSGD_iter=2, min_compression_rate=1.1)
    ddp.register_comm_hook(st, batched_powerSGD_hook if batched else powerSGD_hook)
    base = _mlp()
    for it, (x, y, xs, ys) in enumerate(_data(world, rank, 5)):
        m.zero_grad()
        base.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        F.cross_entropy(base(x), y).backward()
        # grads identical across ranks (compressed or not)
        from distributeddataparallel_amd import distributed as d

        for p in m.parameters():
            r = p.grad.clone()
            d.broadcast(r, 0)
            torch.testing.assert_close(r, p.grad)
        if it < 2:  # vanilla warm-up phase == exact allreduce
            for a, b in zip(m.parameters(), base.parameters()):
                torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)
        else:  # low-rank approximation: correlated with the true gradient
            ga = torch.cat([p.grad.flatten() for p in m.parameters()])
            gb = torch.cat([p.grad.flatten() for p in base.parameters()])
            assert F.cosine_similarity(ga, gb, dim=0) > (0.05 if batched else 0.3)
    if not batched:
        assert st.compression_stats()[0] > 1.0


@pytest.mark.parametrize("batched", [False, True])
def test_powersgd(batched):
    run_ranks(_w_powersgd, world=2, args=(batched,))


def _w_quant(rank, world, kind):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.parallel.comm_hooks import quantization_hooks as q

    m, base = _mlp(), _mlp()
    ddp = xddp.DDP(m)
    ddp.register_comm_hook(None, q.quantization_pertensor_hook if kind == "tensor" else q.quantization_perchannel_hook)
    for x, y, xs, ys in _data(world, rank, 2):
        m.zero_grad()
        base.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        F.cross_entropy(base(x), y).backward()
        for a, b in zip(m.parameters(), base.parameters()):
            scale = b.grad.abs().max().item() + 1e-9
            assert (a.grad - b.grad).abs().max().item() < 0.05 * scale + 1e-4


@pytest.mark.parametrize("kind", ["tensor", "channel"])
def test_quantization_hooks(kind):
    run_ranks(_w_quant, world=2, args=(kind,))


def _w_post_local(rank, world):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as d
    from distributeddataparallel_amd.parallel.comm_hooks.post_localSGD_hook import (PeriodicModelAverager,
                                                                                      PostLocalSGDState,
                                                                                      post_localSGD_hook)

    m = _mlp()
    ddp = xddp.DDP(m)
    sub = d.new_group([rank]) if False else None
    groups = [d.new_group([r]) for r in range(world)]  # every rank creates every group
    st = PostLocalSGDState(process_group=None, subgroup=groups[rank], start_localSGD_iter=2)
    ddp.register_comm_hook(st, post_localSGD_hook)
    avg = PeriodicModelAverager(period=2, warmup_steps=2)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    for it, (x, y, xs, ys) in enumerate(_data(world, rank, 4, seed=5 + rank)):
        opt.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        opt.step()
        avg.average_parameters(m.parameters())
    # step index 2 was an averaging step and step 3 a local one: after the loop params differ,
    # then one more averaging makes them identical
    avg.step = 2
    avg.average_parameters(m.parameters())
    for p in m.parameters():
        r = p.detach().clone()
        d.broadcast(r, 0)
        torch.testing.assert_close(r, p.detach())


def test_post_local_sgd_and_model_averager():
    run_ranks(_w_post_local, world=2)


def _w_fused_optim(rank, world):
    import distributeddataparallel_amd as xddp

    m, base = _mlp(), _mlp()
    ddp = xddp.DDP(m)
    ddp._register_fused_optim(torch.optim.SGD, lr=0.1)
    bopt = torch.optim.SGD(base.parameters(), lr=0.1)
    for x, y, xs, ys in _data(world, rank, 3):
        F.cross_entropy(ddp(xs), ys).backward()  # optimizer runs inside the comm hook
        bopt.zero_grad()
        F.cross_entropy(base(x), y).backward()
        bopt.step()
        m.zero_grad()
    for a, b in zip(m.parameters(), base.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_optimizer_in_backward_hook():
    run_ranks(_w_fused_optim, world=2)


def _w_syncbn(rank, world):
    from distributeddataparallel_amd.parallel.sync_batchnorm import SyncBatchNorm

    torch.manual_seed(0)
    net = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.ReLU())
    ref = nn.Sequential(nn.Conv2d(3, 8, 3), nn.BatchNorm2d(8), nn.ReLU())
    ref.load_state_dict(net.state_dict())
    net = SyncBatchNorm.convert_sync_batchnorm(net)
    assert isinstance(net[1], SyncBatchNorm)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(4 * world, 3, 10, 10, generator=g) * 3 + 1
    xs = x[rank * 4:(rank + 1) * 4].clone().requires_grad_()
    xr = x.clone().requires_grad_()
    ys = net(xs)
    yr = ref(xr)
    torch.testing.assert_close(ys, yr[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(net[1].running_mean, ref[1].running_mean, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(net[1].running_var, ref[1].running_var, rtol=1e-5, atol=1e-6)
    gy = torch.randn(yr.shape, generator=g)
    ys.backward(gy[rank * 4:(rank + 1) * 4])
    yr.backward(gy)
    torch.testing.assert_close(xs.grad, xr.grad[rank * 4:(rank + 1) * 4], rtol=1e-4, atol=1e-5)
    # weight grads are local (DDP all-reduces them); their sum over ranks == full-batch grad
    from distributeddataparallel_amd import distributed as d

    wg = net[1].weight.grad.clone()
    d.all_reduce(wg)
    torch.testing.assert_close(wg, ref[1].weight.grad, rtol=1e-4, atol=1e-5)


def test_sync_batchnorm():
    run_ranks(_w_syncbn, world=2)
