"""DDP behaviour on the native CPU backend, W=2/3 processes.

Oracles: (a) a single-process model trained on the global batch (reference stack's
``_test_DDP_niter`` pattern), and (b) ``torch.nn.parallel.DistributedDataParallel`` over
gloo, run in the same processes on the same data.
"""
import os

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from _dist_utils import run_ranks


def _torch_pg(rank, world):
    import torch.distributed as tdist

    if not tdist.is_initialized():
        tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{os.environ['XDDP_TEST_TORCH_PORT']}",
                                 rank=rank, world_size=world)
    return tdist


def _mlp():
    from distributeddataparallel_amd.models import MLP

    torch.manual_seed(0)
    return MLP(784, 64, 10)


def _batches(world, n, per_rank=8, seed=1):
    g = torch.Generator().manual_seed(seed)
    return [(torch.randn(per_rank * world, 1, 28, 28, generator=g), torch.randint(0, 10, (per_rank * world,), generator=g))
            for _ in range(n)]


def _shard(t, rank, world):
    n = t.shape[0] // world
    return t[rank * n:(rank + 1) * n]


# --------------------------------------------------------------------------------------------
def _w_parity(rank, world, grad_as_view, bucket_cap, rebind=False):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    base = _mlp()
    m1, m2, m3 = _mlp(), _mlp(), _mlp()
    ddp = xddp.DDP(m1, gradient_as_bucket_view=grad_as_view, bucket_cap_mb=bucket_cap)
    tddp = torch.nn.parallel.DistributedDataParallel(m2, gradient_as_bucket_view=grad_as_view)
    opts = [torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9) for m in (m1, m2, base)]
    for it, (x, y) in enumerate(_batches(world, 5)):
        xs, ys = _shard(x, rank, world), _shard(y, rank, world)
        for o in opts:
            o.zero_grad()
        if rebind and it == 2:
            ddp._rebind_grad_accumulators()  # what the HIP-graph helper does before capture
        F.cross_entropy(ddp(xs), ys).backward()
        F.cross_entropy(tddp(xs), ys).backward()
        F.cross_entropy(base(x), y).backward()
        for a, b, c in zip(m1.parameters(), m2.parameters(), base.parameters()):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-7)
            torch.testing.assert_close(a.grad, c.grad, rtol=1e-5, atol=1e-6)
        for o in opts:
            o.step()
    for a, c in zip(m1.parameters(), base.parameters()):
        torch.testing.assert_close(a, c, rtol=1e-5, atol=1e-6)
    if grad_as_view:
        storages = {p.grad.untyped_storage().data_ptr() for p in m1.parameters()}
        assert len(storages) == len(ddp.reducer.bucket_sizes_bytes())
    d = ddp._get_ddp_logging_data()
    assert d["has_rebuilt_buckets"] == "1"
    assert d["world_size"] == str(world)


@pytest.mark.parametrize("grad_as_view", [False, True])
def test_parity_mlp_w2(grad_as_view):
    """BASELINE.json config 1: 2-layer MLP, MNIST-shaped, W=2 on the CPU backend."""
    run_ranks(_w_parity, world=2, args=(grad_as_view, 0.05))


def test_parity_w3_small_buckets():
    run_ranks(_w_parity, world=3, args=(False, 0.01))


def test_parity_after_rebinding_grad_accumulators():
    run_ranks(_w_parity, world=2, args=(True, 0.01, True))


# --------------------------------------------------------------------------------------------
def _w_collectives(rank, world):
    from distributeddataparallel_amd import distributed as d

    t = torch.arange(6, dtype=torch.float32) + rank
    d.all_reduce(t)
    assert torch.equal(t, torch.arange(6, dtype=torch.float32) * world + sum(range(world)))
    t = torch.full((5,), float(rank + 1))
    d.all_reduce(t, op=d.ReduceOp.AVG)
    assert torch.allclose(t, torch.full((5,), (world + 1) / 2))
    for op, fn in [(d.ReduceOp.MAX, max), (d.ReduceOp.MIN, min)]:
        t = torch.tensor([rank * 1.0, -rank * 1.0])
        d.all_reduce(t, op=op)
        assert t[0].item() == fn(range(world)) and t[1].item() == fn(-r for r in range(world))
    t = torch.tensor([rank + 1], dtype=torch.int64)
    d.all_reduce(t, op=d.ReduceOp.PRODUCT)
    import math

    assert t.item() == math.factorial(world)
    bt = torch.full((1000,), rank + 0.5, dtype=torch.bfloat16)
    d.all_reduce(bt)
    assert torch.allclose(bt.float(), torch.full((1000,), sum(r + 0.5 for r in range(world))), rtol=1e-2)
    b = torch.full((3, 4), float(rank))
    d.broadcast(b, src=world - 1)
    assert torch.all(b == world - 1)
    out = [torch.empty(2) for _ in range(world)]
    d.all_gather(out, torch.tensor([rank, rank * 10.0]))
    for r in range(world):
        assert out[r].tolist() == [r, r * 10.0]
    inp = torch.arange(world * 3, dtype=torch.float32)
    o = torch.empty(3)
    d.reduce_scatter_tensor(o, inp)
    assert torch.equal(o, inp[rank * 3:(rank + 1) * 3] * world)
    a2a_in = torch.arange(world * 2, dtype=torch.float32) + 100 * rank
    a2a_out = torch.empty(world * 2)
    d.all_to_all_single(a2a_out, a2a_in)
    for r in range(world):
        assert a2a_out[r * 2:(r + 1) * 2].tolist() == [100 * r + rank * 2, 100 * r + rank * 2 + 1]
    if rank == 0:
        d.send(torch.tensor([42.0]), dst=1)
    elif rank == 1:
        x = torch.zeros(1)
        d.recv(x, src=0)
        assert x.item() == 42.0
    d.barrier()
    objs = [None] * world
    d.all_gather_object(objs, {"rank": rank})
    assert [o["rank"] for o in objs] == list(range(world))
    lst = [rank, "x"] if rank == 0 else [None, None]
    d.broadcast_object_list(lst, src=0)
    assert lst == [0, "x"]
    # async + future
    w = d.get_default_group().allreduce(torch.ones(4))
    fut = w.get_future()
    assert torch.equal(fut.wait()[0], torch.full((4,), float(world)))
    # sub-group of even ranks
    g = d.new_group([r for r in range(world) if r % 2 == 0])
    if rank % 2 == 0:
        t = torch.ones(2)
        d.all_reduce(t, group=g)
        assert t[0].item() == len([r for r in range(world) if r % 2 == 0])
    recs = d.get_default_group().flight_records()
    assert len(recs) > 10 and all(r["state"] in ("completed", "scheduled") for r in recs)


@pytest.mark.parametrize("world", [2, 3])
def test_collectives(world):
    run_ranks(_w_collectives, world=world)


# --------------------------------------------------------------------------------------------
def _w_no_sync(rank, world):
    import distributeddataparallel_amd as xddp

    base, m = _mlp(), _mlp()
    ddp = xddp.DDP(m)
    batches = _batches(world, 4)
    for i, (x, y) in enumerate(batches):
        xs, ys = _shard(x, rank, world), _shard(y, rank, world)
        if i % 2 == 0:
            with ddp.no_sync():
                F.cross_entropy(ddp(xs), ys).backward()
            F.cross_entropy(base(x), y).backward()
            # local only: differs from the global-batch grads
            if world > 1:
                assert any(not torch.allclose(a.grad, b.grad) for a, b in zip(m.parameters(), base.parameters()))
        else:
            F.cross_entropy(ddp(xs), ys).backward()
            F.cross_entropy(base(x), y).backward()
            for a, b in zip(m.parameters(), base.parameters()):
                torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)
            for p in list(m.parameters()) + list(base.parameters()):
                p.grad = None
    # no_sync + no_grad leaves no residue
    with ddp.no_sync(), torch.no_grad():
        ddp(batches[0][0][:2])
    assert ddp.reducer.finalized()


def test_no_sync_accumulation():
    run_ranks(_w_no_sync, world=2)


# --------------------------------------------------------------------------------------------
class _Branchy(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = nn.Linear(10, 10)
        self.b = nn.Linear(10, 10)
        self.head = nn.Linear(10, 2)

    def forward(self, x, use_b: bool):
        h = F.relu(self.a(x))
        if use_b:
            h = h + F.relu(self.b(x))
        return self.head(h)


def _w_find_unused(rank, world, static):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _Branchy(), _Branchy()
    ddp = xddp.DDP(m1, find_unused_parameters=not static, static_graph=static)
    tddp = torch.nn.parallel.DistributedDataParallel(m2, find_unused_parameters=not static, static_graph=static)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(3 + rank)
    for it in range(5):
        x = torch.randn(4, 10, generator=g)
        use_b = (it % 2 == 0) if not static else False
        if not static and rank == 1:
            use_b = True  # rank 1 always uses b: b is globally used every iteration
        o1.zero_grad()
        o2.zero_grad()
        ddp(x, use_b).sum().backward()
        tddp(x, use_b).sum().backward()
        for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
            if b.grad is None:
                assert a.grad is None or torch.all(a.grad == 0), n
            else:
                torch.testing.assert_close(a.grad, b.grad, rtol=1e-6, atol=1e-7, msg=n)
        o1.step()
        o2.step()


def test_find_unused_parameters():
    run_ranks(_w_find_unused, world=2, args=(False,))


def test_static_graph_with_unused_branch():
    run_ranks(_w_find_unused, world=2, args=(True,))


def _w_unused_error(rank, world):
    import distributeddataparallel_amd as xddp

    ddp = xddp.DDP(_Branchy())
    x = torch.randn(4, 10)
    ddp(x, False).sum().backward()
    try:
        ddp(x, False).sum().backward()
    except RuntimeError as e:
        assert "Expected to have finished reduction in the prior iteration" in str(e)
        assert "b.weight" in str(e)
    else:
        raise AssertionError("expected an unused-parameter error")


def test_unused_params_error_message():
    run_ranks(_w_unused_error, world=2)


# --------------------------------------------------------------------------------------------
class _BNNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 8, 3)
        self.bn = nn.BatchNorm2d(8)
        self.fc = nn.Linear(8, 2)

    def forward(self, x):
        return self.fc(F.relu(self.bn(self.conv(x))).mean((2, 3)))


def _w_buffers_and_init_sync(rank, world):
    import distributeddataparallel_amd as xddp

    torch.manual_seed(100 + rank)  # different init per rank: ctor must broadcast rank 0's
    m = _BNNet()
    ddp = xddp.DDP(m)
    from distributeddataparallel_amd import distributed as d

    for p in m.parameters():
        ref = p.detach().clone()
        d.broadcast(ref, 0)
        assert torch.equal(ref, p.detach())
    for _ in range(3):
        ddp(torch.randn(4, 3, 8, 8) + rank).sum().backward()
    # running stats were broadcast from rank 0 before each forward: after a final forward from
    # identical rank-0 buffers, compare (rank 0's post-forward stats are what everyone saw)
    rm = m.bn.running_mean.clone()
    d.broadcast(rm, 0)
    # state_dict layout == torch DDP's
    tdist = _torch_pg(rank, world)
    tddp = torch.nn.parallel.DistributedDataParallel(_BNNet())
    assert list(ddp.state_dict().keys()) == list(tddp.state_dict().keys())
    assert all(k.startswith("module.") for k in ddp.state_dict())


def test_buffers_init_sync_and_state_dict_layout():
    run_ranks(_w_buffers_and_init_sync, world=2)


def _w_buffer_sync(rank, world):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as d

    m = _BNNet()
    ddp = xddp.DDP(m)
    with torch.no_grad():
        m.bn.running_mean.fill_(float(rank + 7))
    ddp(torch.zeros(2, 3, 8, 8))  # pre-forward broadcast from rank 0, then this forward's EMA
    assert m.bn.running_mean.allclose(m.bn.running_mean.new_full((8,), 7.0 * 0.9) + 0.1 * m.bn.running_mean.new_tensor(
        F.conv2d(torch.zeros(2, 3, 8, 8), m.conv.weight, m.conv.bias).mean((0, 2, 3))))
    m2 = _BNNet()
    ddp2 = xddp.DDP(m2, broadcast_buffers=False)
    with torch.no_grad():
        m2.bn.running_mean.fill_(float(rank + 7))
        ddp2.eval()
        ddp2(torch.zeros(1, 3, 8, 8))
    assert m2.bn.running_mean[0].item() == rank + 7


def test_buffer_broadcast_every_forward():
    run_ranks(_w_buffer_sync, world=2)


# --------------------------------------------------------------------------------------------
def _w_join(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _mlp(), _mlp()
    ddp = xddp.DDP(m1)
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    n = 3 + 2 * rank  # uneven inputs
    batches = _batches(1, n, per_rank=4, seed=10 + rank)
    with ddp.join():
        for x, y in batches:
            o1.zero_grad()
            F.cross_entropy(ddp(x), y).backward()
            o1.step()
    with tddp.join():
        for x, y in batches:
            o2.zero_grad()
            F.cross_entropy(tddp(x), y).backward()
            o2.step()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    from distributeddataparallel_amd import distributed as d

    for p in m1.parameters():
        r = p.detach().clone()
        d.broadcast(r, 0)
        assert torch.equal(r, p.detach())


def test_join_uneven_inputs_matches_torch():
    run_ranks(_w_join, world=2)


# --------------------------------------------------------------------------------------------
def _w_hooks(rank, world, hook_name):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.parallel.comm_hooks import debugging_hooks, default_hooks

    base, m = _mlp(), _mlp()
    ddp = xddp.DDP(m)
    hook = {"allreduce": default_hooks.allreduce_hook, "fp16": default_hooks.fp16_compress_hook,
            "bf16": default_hooks.bf16_compress_hook, "noop": debugging_hooks.noop_hook,
            "fp16_wrap": default_hooks.fp16_compress_wrapper(default_hooks.allreduce_hook)}[hook_name]
    ddp.register_comm_hook(None, hook)
    with pytest.raises(RuntimeError):
        ddp.register_comm_hook(None, hook)
    for x, y in _batches(world, 3):
        xs, ys = _shard(x, rank, world), _shard(y, rank, world)
        m.zero_grad()
        base.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        F.cross_entropy(base(x), y).backward()
        for a, b in zip(m.parameters(), base.parameters()):
            if hook_name == "noop":
                continue
            tol = 1e-5 if hook_name == "allreduce" else 2e-2
            torch.testing.assert_close(a.grad, b.grad, rtol=tol, atol=tol)


@pytest.mark.parametrize("hook_name", ["allreduce", "fp16", "bf16", "noop", "fp16_wrap"])
def test_comm_hooks(hook_name):
    run_ranks(_w_hooks, world=2, args=(hook_name,))


def _w_comm_dtype(rank, world):
    import distributeddataparallel_amd as xddp

    base, m = _mlp(), _mlp()
    ddp = xddp.DDP(m, comm_dtype=torch.bfloat16)
    for x, y in _batches(world, 2):
        xs, ys = _shard(x, rank, world), _shard(y, rank, world)
        m.zero_grad()
        base.zero_grad()
        F.cross_entropy(ddp(xs), ys).backward()
        F.cross_entropy(base(x), y).backward()
        for a, b in zip(m.parameters(), base.parameters()):
            scale = b.grad.abs().max().item() + 1e-12
            assert (a.grad - b.grad).abs().max().item() < 2e-2 * scale


def test_builtin_bf16_comm_dtype():
    run_ranks(_w_comm_dtype, world=2)


# --------------------------------------------------------------------------------------------
def _w_mismatch(rank, world):
    import distributeddataparallel_amd as xddp

    m = nn.Linear(4, 4) if rank == 0 else nn.Linear(4, 5)
    try:
        xddp.DDP(m)
    except RuntimeError as e:
        assert "same model across all ranks" in str(e) or "sizes" in str(e)
    else:
        raise AssertionError("expected a shape-mismatch error")


def test_model_mismatch_detected():
    run_ranks(_w_mismatch, world=2)


def _w_pickle(rank, world):
    import io

    import distributeddataparallel_amd as xddp

    ddp = xddp.DDP(_mlp())
    buf = io.BytesIO()
    torch.save(ddp, buf)
    buf.seek(0)
    ddp2 = torch.load(buf, weights_only=False)  # our own object, written by this test
    x, y = _batches(world, 1)[0]
    F.cross_entropy(ddp2(_shard(x, rank, world)), _shard(y, rank, world)).backward()
    assert all(p.grad is not None for p in ddp2.parameters())


def test_pickle_roundtrip():
    run_ranks(_w_pickle, world=2)
