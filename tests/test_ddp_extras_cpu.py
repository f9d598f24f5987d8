"""DDP options beyond the reference's default call on the CPU backend."""
import pytest
import torch
import torch.nn.functional as F

from _dist_utils import run_ranks
from test_ddp_cpu import _batches, _mlp, _shard, _torch_pg


def _w_delay(rank, world, all_params):
    import distributeddataparallel_amd as xddp

    m1, base = _mlp(), _mlp()
    named1 = list(m1.named_parameters())
    k = len(named1) if all_params else 2  # delay the first layer (its grads are ready last)
    ddp = xddp.DDP(m1, delay_all_reduce_named_params=named1[:k], param_to_hook_all_reduce=named1[0][1])
    assert ddp._delay_all_reduce_all_params == all_params
    o1 = torch.optim.SGD(m1.parameters(), lr=0.05)
    o2 = torch.optim.SGD(base.parameters(), lr=0.05)
    for it, (x, y) in enumerate(_batches(world, 4)):
        xs, ys = _shard(x, rank, world), _shard(y, rank, world)
        o1.zero_grad(set_to_none=(it % 2 == 0))
        o2.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        F.cross_entropy(base(x), y).backward()  # oracle: one process on the global batch
        for a, b in zip(m1.parameters(), base.parameters()):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)
        o1.step()
        o2.step()
    for a, b in zip(m1.parameters(), base.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("all_params", [False, True])
def test_delay_all_reduce_named_params_matches_torch(all_params):
    run_ranks(_w_delay, world=2, args=(all_params,))


def _w_mixed_precision(rank, world):
    from types import SimpleNamespace

    from torch.func import functional_call

    import distributeddataparallel_amd as xddp

    m1, base = _mlp(), _mlp()
    mp = SimpleNamespace(param_dtype=torch.bfloat16, reduce_dtype=torch.float32, buffer_dtype=None)
    ddp = xddp.DDP(m1, mixed_precision=mp)
    for x, y in _batches(world, 3):
        xs, ys = _shard(x, rank, world), _shard(y, rank, world)
        ddp.zero_grad()
        base.zero_grad()
        out = ddp(xs)
        assert out.dtype == torch.bfloat16
        F.cross_entropy(out.float(), ys).backward()
        # oracle: the same bf16-parameter forward on the global batch, grads w.r.t. fp32 leaves
        names = [n for n, _ in base.named_parameters()]
        casted = {n: p.to(torch.bfloat16) for n, p in base.named_parameters()}
        F.cross_entropy(functional_call(base, casted, (x.to(torch.bfloat16),)).float(), y).backward()
        for (n, a), b in zip(m1.named_parameters(), base.parameters()):
            assert a.dtype == torch.float32 and a.grad.dtype == torch.float32
            torch.testing.assert_close(a.grad, b.grad, rtol=3e-2, atol=3e-3)
        assert names


def test_mixed_precision_params_bf16_grads_fp32():
    run_ranks(_w_mixed_precision, world=2)
