"""Round-2 DDP API behaviours on the native CPU backend, each against torch DDP over gloo in the
same processes (SURVEY.md §4.2 behaviour checklist; VERDICT r1 "Next round" #8):

* join(divide_by_initial_world_size=False) must not leak its divide factor into later steps;
* join + no_sync on the non-joined ranks must not mis-pair collectives;
* a rank that joins before finishing one iteration still follows the bucket rebuild;
* sparse gradients (nn.Embedding(sparse=True));
* skip_all_reduce_unused_params;
* _register_buffer_comm_hook (PRE/POST forward, futures awaited at end of backward);
* device_mesh (1-D);
* uneven all_to_all_single splits; non-blocking Work.get_future; Work.wait(timeout).
"""
import datetime

import torch
import torch.nn as nn
import torch.nn.functional as F

from _dist_utils import run_ranks
from test_ddp_cpu import _batches, _mlp, _shard, _torch_pg


def _assert_params_equal(m1, m2, rtol=1e-5, atol=1e-6):
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=rtol, atol=atol)


# --------------------------------------------------------------------------------------------
def _w_join_divide_reset(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _mlp(), _mlp()
    ddp = xddp.DDP(m1)
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    uneven = _batches(1, 2 + 2 * rank, per_rank=4, seed=20 + rank)
    after = _batches(1, 3, per_rank=4, seed=40 + rank)
    for model, opt, wrap in ((ddp, o1, ddp), (tddp, o2, tddp)):
        with wrap.join(divide_by_initial_world_size=False):
            for x, y in uneven:
                opt.zero_grad()
                F.cross_entropy(model(x), y).backward()
                opt.step()
        # after the join block every rank trains again: grads must be the world mean
        for x, y in after:
            opt.zero_grad()
            F.cross_entropy(model(x), y).backward()
            opt.step()
    _assert_params_equal(m1, m2)


def test_join_divide_factor_does_not_leak():
    run_ranks(_w_join_divide_reset, world=2)


# --------------------------------------------------------------------------------------------
def _w_join_no_sync(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _mlp(), _mlp()
    ddp = xddp.DDP(m1)
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    batches = _batches(1, 2 + 4 * rank, per_rank=4, seed=60 + rank)
    for model, opt in ((ddp, o1), (tddp, o2)):
        with model.join():
            for i, (x, y) in enumerate(batches):
                if i % 2 == 0:  # accumulate locally on even steps
                    with model.no_sync():
                        F.cross_entropy(model(x), y).backward()
                else:
                    F.cross_entropy(model(x), y).backward()
                    opt.step()
                    opt.zero_grad()
    _assert_params_equal(m1, m2)


def test_join_with_no_sync_iterations():
    run_ranks(_w_join_no_sync, world=2)


# --------------------------------------------------------------------------------------------
def _w_join_before_first_iteration(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _mlp(), _mlp()
    ddp = xddp.DDP(m1)
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    batches = _batches(1, 0 if rank == 1 else 4, per_rank=4, seed=80 + rank)  # rank 1: no inputs at all
    for model, opt in ((ddp, o1), (tddp, o2)):
        with model.join():
            for x, y in batches:
                opt.zero_grad()
                F.cross_entropy(model(x), y).backward()
                opt.step()
    _assert_params_equal(m1, m2)
    assert ddp._get_ddp_logging_data()["has_rebuilt_buckets"] == "1"


def test_join_rank_without_any_input_follows_rebuild():
    run_ranks(_w_join_before_first_iteration, world=2)


# --------------------------------------------------------------------------------------------
class _EmbNet(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(3)
        self.emb = nn.Embedding(50, 16, sparse=True)
        self.fc = nn.Linear(16, 4)

    def forward(self, idx):
        return self.fc(self.emb(idx).mean(1))


def _w_sparse(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _EmbNet(), _EmbNet()
    ddp = xddp.DDP(m1)
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.5), torch.optim.SGD(m2.parameters(), lr=0.5)
    g = torch.Generator().manual_seed(100 + rank)
    for it in range(4):
        idx = torch.randint(0, 50, (6, 5), generator=g)
        y = torch.randint(0, 4, (6,), generator=g)
        for model, opt in ((ddp, o1), (tddp, o2)):
            opt.zero_grad()
            F.cross_entropy(model(idx), y).backward()
            if model is ddp:
                assert m1.emb.weight.grad.is_sparse
            opt.step()
        _assert_params_equal(m1, m2)


def test_sparse_embedding_gradients_match_torch():
    run_ranks(_w_sparse, world=2)


# --------------------------------------------------------------------------------------------
class _TwoHeads(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(4)
        self.body = nn.Linear(8, 8)
        self.used = nn.Linear(8, 3)
        self.unused = nn.Linear(8, 3)

    def forward(self, x):
        return self.used(torch.relu(self.body(x)))


def _w_skip_unused(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2 = _TwoHeads(), _TwoHeads()
    # small caps: the unused head lands in a bucket of its own, which is then skipped
    ddp = xddp.DDP(m1, find_unused_parameters=True, skip_all_reduce_unused_params=True, bucket_cap_mb=0.0001,
                   first_bucket_cap_mb=0.0001)
    tddp = torch.nn.parallel.DistributedDataParallel(m2, find_unused_parameters=True)
    o1, o2 = torch.optim.SGD(m1.parameters(), lr=0.1), torch.optim.SGD(m2.parameters(), lr=0.1)
    g = torch.Generator().manual_seed(7 + rank)
    n0 = ddp.process_group.comm.num_collectives()
    for _ in range(3):
        x, y = torch.randn(4, 8, generator=g), torch.randint(0, 3, (4,), generator=g)
        for model, opt in ((ddp, o1), (tddp, o2)):
            opt.zero_grad()
            F.cross_entropy(model(x), y).backward()
            opt.step()
    _assert_params_equal(m1, m2)
    assert m1.unused.weight.grad is None
    ddp2 = xddp.DDP(_TwoHeads(), find_unused_parameters=True, bucket_cap_mb=0.0001, first_bucket_cap_mb=0.0001)
    n1 = ddp2.process_group.comm.num_collectives()
    x = torch.randn(4, 8)
    F.cross_entropy(ddp2(x), torch.zeros(4, dtype=torch.long)).backward()
    n_full = ddp2.process_group.comm.num_collectives() - n1
    n2 = ddp.process_group.comm.num_collectives()
    F.cross_entropy(ddp(x), torch.zeros(4, dtype=torch.long)).backward()
    n_skip = ddp.process_group.comm.num_collectives() - n2
    assert n_skip < n_full, (n_skip, n_full)


def test_skip_all_reduce_unused_params():
    run_ranks(_w_skip_unused, world=2)


# --------------------------------------------------------------------------------------------
class _BufNet(nn.Module):
    """Buffers that are not saved for backward (like the reference test's NetWithBuffers)."""

    def __init__(self):
        super().__init__()
        torch.manual_seed(5)
        self.fc = nn.Linear(6, 6)
        self.register_buffer("running_mean", torch.zeros(6))
        self.register_buffer("steps", torch.zeros((), dtype=torch.long))

    def forward(self, x):
        y = self.fc(x)
        with torch.no_grad():
            self.running_mean.mul_(0.9).add_(0.1 * y.mean(0))
            self.steps += 1
        return y


def _w_buffer_hook(rank, world, location):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.parallel.distributed import BufferCommHookLocation

    m = _BufNet()
    ddp = xddp.DDP(m)
    calls = []

    def hook(state, named_buffers):
        calls.append(sorted(named_buffers))
        futs = []
        for n, b in named_buffers.items():
            if b.is_floating_point():
                futs.append(xdist.all_reduce(b, op=xdist.ReduceOp.AVG, async_op=True).get_future())
        return futs

    ddp._register_buffer_comm_hook(None, hook, getattr(BufferCommHookLocation, location))
    g = torch.Generator().manual_seed(rank)
    for _ in range(2):
        x = torch.randn(8, 6, generator=g) + rank
        ddp(x).sum().backward()
    assert len(calls) == 2 and calls[0] == ["running_mean", "steps"]
    if location == "PRE_FORWARD":  # the forward after the hook updates buffers locally again
        with torch.no_grad():
            m.running_mean.zero_()
            for f in hook(None, ddp.named_module_buffers):
                f.wait()
    # buffers are the average over ranks (not rank 0's copy): equal everywhere
    r = m.running_mean.clone()
    xdist.broadcast(r, 0)
    torch.testing.assert_close(r, m.running_mean)
    assert m.steps.item() == 2


def test_buffer_comm_hook_post_forward():
    run_ranks(_w_buffer_hook, world=2, args=("POST_FORWARD",))


def test_buffer_comm_hook_pre_forward():
    run_ranks(_w_buffer_hook, world=2, args=("PRE_FORWARD",))


# --------------------------------------------------------------------------------------------
def _w_mesh(rank, world):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist

    class Mesh:
        ndim = 1

        def get_group(self, mesh_dim=0):
            return xdist.get_default_group()

    base, m = _mlp(), _mlp()
    ddp = xddp.DDP(m, device_mesh=Mesh())
    assert ddp.process_group is xdist.get_default_group()
    ob, om = torch.optim.SGD(base.parameters(), lr=0.1), torch.optim.SGD(m.parameters(), lr=0.1)
    for x, y in _batches(world, 2):
        for model, opt, xs, ys in ((ddp, om, _shard(x, rank, world), _shard(y, rank, world)), (base, ob, x, y)):
            opt.zero_grad()
            F.cross_entropy(model(xs), ys).backward()
            opt.step()
    _assert_params_equal(m, base)


def test_device_mesh_1d():
    run_ranks(_w_mesh, world=2)


# --------------------------------------------------------------------------------------------
def _w_alltoall_uneven(rank, world):
    from distributeddataparallel_amd import distributed as xdist

    tdist = _torch_pg(rank, world)
    # rank r sends (r + 1 + dst) rows to rank dst
    in_splits = [rank + 1 + d for d in range(world)]
    out_splits = [s + 1 + rank for s in range(world)]
    inp = torch.cat([torch.full((n, 3), float(100 * rank + d)) for d, n in enumerate(in_splits)])
    out = torch.empty(sum(out_splits), 3)
    xdist.all_to_all_single(out, inp, output_split_sizes=out_splits, input_split_sizes=in_splits)
    ref = torch.empty_like(out)
    tdist.all_to_all_single(ref, inp, output_split_sizes=out_splits, input_split_sizes=in_splits)
    torch.testing.assert_close(out, ref)


def test_all_to_all_single_uneven_splits():
    run_ranks(_w_alltoall_uneven, world=3)


def _w_future(rank, world):
    from distributeddataparallel_amd import distributed as xdist

    t = torch.full((1 << 16,), float(rank + 1))
    work = xdist.all_reduce(t, async_op=True)
    fut = work.get_future()  # must not block
    res = fut.wait()
    got = res[0] if isinstance(res, (list, tuple)) else res
    assert torch.all(got == sum(range(1, world + 1)))
    # wait(timeout) raises while the partner has not joined; the collective stays usable
    import time

    if rank == 0:
        w = xdist.all_reduce(torch.ones(4), async_op=True)
        t0 = time.monotonic()
        try:
            w.wait(timeout=datetime.timedelta(seconds=0.3))
            raised = False
        except RuntimeError:
            raised = True
        assert raised and time.monotonic() - t0 < 1.0
        w.wait()
    else:
        time.sleep(1.5)  # late partner of rank 0's pending all-reduce
        xdist.all_reduce(torch.ones(4))
    xdist.barrier()


def test_work_future_and_wait_timeout():
    run_ranks(_w_future, world=2)


def _w_monitored_barrier(rank, world):
    import time

    from distributeddataparallel_amd import distributed as dist

    # back-to-back barriers with a slow rank: a fast rank must never pass barrier k+1 early
    arrive = []
    for k in range(4):
        if rank == 1:
            time.sleep(0.2)
        dist.monitored_barrier(timeout=datetime.timedelta(seconds=20))
        arrive.append(time.time())
    from distributeddataparallel_amd.distributed.c10d import _resolve

    store = _resolve(None).store
    # publish rank 1's exit times; rank 0 must leave every barrier after rank 1 reached it
    store.set(f"mb_test/{rank}", ",".join(f"{t:.6f}" for t in arrive))
    dist.barrier()
    if rank == 0:
        raw = store.get("mb_test/1")
        other = [float(t) for t in (raw.decode() if isinstance(raw, bytes) else raw).split(",")]
        for k in range(4):
            assert arrive[k] >= other[k] - 0.15, (k, arrive, other)
    # a missing rank is named
    if rank == 0:
        try:
            dist.monitored_barrier(timeout=datetime.timedelta(seconds=0.5), wait_all_ranks=True)
        except RuntimeError as e:
            assert "missing ranks [1]" in str(e), str(e)
        else:
            raise AssertionError("expected a timeout")
    dist.barrier()


def test_monitored_barrier_generations_and_missing_ranks():
    run_ranks(_w_monitored_barrier, world=2)


# --------------------------------------------------------------------------------------------
def _w_python_reducer(rank, world):
    import distributeddataparallel_amd as xddp

    tdist = _torch_pg(rank, world)
    m1, m2, m3 = _mlp(), _mlp(), _mlp()
    ddp = xddp.DDP(m1, python_reducer=True)
    assert ddp._use_python_reducer and len(ddp._accum_grad_hooks) == len(list(m1.parameters()))
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    seen = []

    def hook(state, grad_and_param):  # the compiled-mode comm-hook protocol: (grad, param)
        g, p = grad_and_param
        seen.append(p.shape)
        w = state.allreduce(g, xddp.distributed.ReduceOp.AVG)
        w.wait()

    ddp_h = xddp.DDP(m3, python_reducer=True)
    ddp_h.register_comm_hook(ddp_h.process_group, hook)
    opts = [torch.optim.SGD(m.parameters(), lr=0.1) for m in (m1, m2, m3)]
    for x, y in _batches(1, 3, per_rank=4, seed=80 + rank):
        for model, opt in zip((ddp, tddp, ddp_h), opts):
            opt.zero_grad()
            F.cross_entropy(model(x), y).backward()
            opt.step()
        with ddp.no_sync():  # no_sync: local accumulation only
            F.cross_entropy(ddp(x), y).backward()
        g_local = [p.grad.clone() for p in m1.parameters()]
        opts[0].zero_grad()
        for p, g in zip(m1.parameters(), g_local):
            assert g.abs().sum() > 0
    _assert_params_equal(m1, m2)
    _assert_params_equal(m3, m2)
    assert len(seen) == 3 * len(list(m3.parameters()))


def test_python_reducer_matches_torch_ddp():
    """T6k: the compiled-autograd "python reducer" mode (per-parameter post-accumulate-grad
    all-reduce) trains identically to torch DDP; comm hooks get (grad, param)."""
    run_ranks(_w_python_reducer, world=2)


# --------------------------------------------------------------------------------------------
def _w_overlapped_optimizer(rank, world, schedule):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.optim import FusedAdamW

    m1, m2 = _mlp(), _mlp()
    d1 = xddp.DDP(m1, bucket_cap_mb=0.001, first_bucket_cap_mb=0.001)  # several buckets
    d2 = xddp.DDP(m2)
    # tail chunks of 16,384 fp32 elements: the last bucket (fc1's weight + bias, 50,240 elements)
    # is all-reduced as 4 collectives and updated slice by slice
    d1.register_overlapped_optimizer(o1 := FusedAdamW(m1.parameters(), lr=1e-2, weight_decay=0.1),
                                     schedule=schedule, tail_chunk_bytes=16384 * 4)
    o2 = FusedAdamW(m2.parameters(), lr=1e-2, weight_decay=0.1)
    log = []
    pg = d1.process_group
    orig_ar, orig_slices = pg.allreduce, o1.step_slices
    pg.allreduce = lambda t, *a, **k: (log.append(("ar", t.numel())), orig_ar(t, *a, **k))[1]
    o1.step_slices = lambda pieces: (log.append(("step", sum(hi - lo for _, _, lo, hi in pieces))),
                                     orig_slices(pieces))[1]
    for x, y in _batches(1, 4, per_rank=4, seed=90 + rank):
        o1.zero_grad()
        log.clear()
        F.cross_entropy(d1(x), y).backward()  # updated inside backward
        o2.zero_grad()
        F.cross_entropy(d2(x), y).backward()
        # .grad after the overlapped backward holds the reduced gradient, as with plain DDP
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            assert torch.equal(p1.grad, p2.grad)
        o2.step()
    pg.allreduce, o1.step_slices = orig_ar, orig_slices
    _assert_params_equal(m1, m2, rtol=0, atol=0)  # bitwise: same all-reduce sums, elementwise AdamW
    nb = len(d1.reducer.bucket_sizes_bytes())
    assert nb >= 2
    ars = [i for i, e in enumerate(log) if e[0] == "ar"]
    steps = [i for i, e in enumerate(log) if e[0] == "step"]
    if schedule == "backward":
        # every bucket's update is issued right after its own all-reduce, one all-reduce per bucket
        assert len(ars) == nb and len(steps) == nb, log
        for b in range(nb):
            assert ars[b] < steps[b] and (b + 1 == nb or steps[b] < ars[b + 1]), log
    else:
        # every collective (nb - 1 buckets + 4 tail chunks) is issued before the first update: the
        # deferred updates run on the side stream while the chunked tail all-reduce is in flight,
        # then the tail's slices, which add up to the whole tail bucket
        assert len(ars) == nb - 1 + 4, log
        assert max(ars) < min(steps), log
        tail_numel = m1.fc1.weight.numel() + m1.fc1.bias.numel()  # the last bucket: fc1's grads
        assert [e[1] for e in log[-4:]] == [16384, 16384, 16384, tail_numel - 3 * 16384], log
        assert d1._overlap_state["last_chunks"] == 4


def test_overlapped_optimizer_matches_step_after_backward():
    """DDP.register_overlapped_optimizer, schedule="backward": the per-bucket FusedAdamW.step_params
    inside backward trains exactly like the usual backward-then-step."""
    run_ranks(_w_overlapped_optimizer, world=2, args=("backward",))


def test_overlapped_optimizer_tail_schedule_chunked_bitwise():
    """schedule="tail" (the default): updates deferred under a chunked tail all-reduce, stepped in
    slices — bitwise equal to the unchunked backward-then-step path."""
    run_ranks(_w_overlapped_optimizer, world=2, args=("tail",))


def test_tail_chunks_ranges():
    from distributeddataparallel_amd.parallel.distributed import tail_chunks

    assert tail_chunks(1000, 4, 1 << 20) == [(0, 1000)]
    r = tail_chunks(525_336_576, 2, 64 << 20)  # Llama-3-8B token embedding, bf16
    assert len(r) == 16 and r[0] == (0, 33_554_432) and r[-1][1] == 525_336_576
    assert all(lo % 4096 == 0 for lo, _ in r) and all(a[1] == b[0] for a, b in zip(r, r[1:]))


def _w_join_buffer_hook(rank, world, location):
    """Uneven inputs + a buffer comm hook: the joined rank must shadow the hook's collectives
    (not a broadcast) at the same point of the iteration."""
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.parallel.distributed import BufferCommHookLocation

    m = _BufNet()
    ddp = xddp.DDP(m)

    def hook(state, named_buffers):
        return [xdist.all_reduce(b, op=xdist.ReduceOp.AVG, async_op=True).get_future()
                for b in named_buffers.values() if b.is_floating_point()]

    ddp._register_buffer_comm_hook(None, hook, getattr(BufferCommHookLocation, location))
    g = torch.Generator().manual_seed(rank)
    n_inputs = 4 if rank == 0 else 1
    with ddp.join():
        for _ in range(n_inputs):
            ddp(torch.randn(8, 6, generator=g) + rank).sum().backward()
    # both ranks still agree afterwards: a healthy collective sequence
    t = torch.tensor([float(rank + 1)])
    xdist.all_reduce(t)
    assert t.item() == 3.0
    assert m.steps.item() == 4  # the final model sync copies the last joiner's buffers


def test_join_with_buffer_comm_hook_post_forward():
    run_ranks(_w_join_buffer_hook, world=2, args=("POST_FORWARD",))


def test_join_with_buffer_comm_hook_pre_forward():
    run_ranks(_w_join_buffer_hook, world=2, args=("PRE_FORWARD",))
