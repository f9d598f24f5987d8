"""Multi-rank DDP on GPU tensors with one MI355X: two ranks share cuda:0.

RCCL refuses two ranks on one device, so these ranks use the native CPU backend, which stages
device tensors through host memory. Everything else is the W=2 GPU path: the Reducer's
device buckets and 1/W pre-division kernels, the bucket rebuild after iteration 0 (rank 0's
order broadcast), buffer broadcast, no_sync accumulation and finalize ordering on HIP streams.
A second test runs the W=1 RCCL communicator with XDDP_RCCL_FORCE_LAUNCH=1, so real RCCL
kernels run on the comm stream (the launch path an 8-GPU job takes).

Oracle: the mean over shards of per-shard gradients, computed locally in each rank on a
parameter-synced replica. That matches DDP even with BatchNorm, whose statistics are per shard.
"""
import os

import pytest
import torch
import torch.nn.functional as F

from _dist_utils import run_ranks

pytestmark = pytest.mark.gpu


def _model():
    from distributeddataparallel_amd.models import SimpleCNN
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    torch.manual_seed(0)
    return SimpleCNN(norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last)


def _w_gpu_parity(rank, world, grad_as_view, accum):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as dist

    torch.cuda.set_device(0)
    # deterministic MIOpen algorithms: DDP must then match the oracle exactly, so any ordering
    # race in staging / bucket copies / finalize shows up as a mismatch instead of noise
    torch.backends.cudnn.deterministic = True
    model, ref = _model(), _model()
    ddp = xddp.DDP(model, device_ids=[0], gradient_as_bucket_view=grad_as_view, bucket_cap_mb=4)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
    g = torch.Generator(device="cuda").manual_seed(7)
    per = 8
    for it in range(4):
        ref.load_state_dict(model.state_dict())
        micro = [(torch.randn(per * world, 3, 32, 32, device="cuda", generator=g).contiguous(
            memory_format=torch.channels_last), torch.randint(0, 10, (per * world,), device="cuda", generator=g))
            for _ in range(accum)]
        opt.zero_grad()
        ref.zero_grad()
        for i, (x, y) in enumerate(micro):
            xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
            if i < accum - 1:
                with ddp.no_sync():
                    F.cross_entropy(ddp(xs), ys).backward()
            else:
                F.cross_entropy(ddp(xs), ys).backward()
            for r in range(world):  # oracle: mean over every rank's shard
                F.cross_entropy(ref(x[r * per:(r + 1) * per]), y[r * per:(r + 1) * per]).div(world).backward()
        for (n, p), q in zip(model.named_parameters(), ref.parameters()):
            scale = q.grad.abs().max().item() + 1e-6
            err = (p.grad - q.grad).abs().max().item()
            assert err <= 1e-6 * scale, f"rank {rank} it {it} {n}: max err {err} (scale {scale})"
        opt.step()
    # replicas stay bit-identical across ranks
    flat = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    allp = torch.empty(world * flat.numel(), device="cuda")
    dist.all_gather_into_tensor(allp, flat)
    allp = allp.view(world, -1)
    assert torch.equal(allp[0], allp[1]), "parameters diverged across ranks"
    # running stats are updated locally by each forward and re-broadcast from rank 0 before the
    # next one (as in torch DDP): sync once, then they must be identical
    ddp._sync_buffers()
    bufs = torch.cat([b.detach().float().reshape(-1) for b in model.buffers()])
    allb = torch.empty(world * bufs.numel(), device="cuda")
    dist.all_gather_into_tensor(allb, bufs)
    assert torch.equal(allb.view(world, -1)[0], allb.view(world, -1)[1]), "buffers diverged across ranks"
    d = ddp._get_ddp_logging_data()
    assert d["has_rebuilt_buckets"] == "1"
    assert ddp.reducer.native_launches() > 0


@pytest.mark.parametrize("grad_as_view,accum", [(False, 1), (True, 2)])
def test_two_ranks_one_gpu_ddp_parity(grad_as_view, accum):
    run_ranks(_w_gpu_parity, world=2, backend="cpu", args=(grad_as_view, accum))


def test_rccl_forced_launch_ddp_steps():
    """W=1 with real RCCL kernels: DDP grads still equal the plain model's (AVG over one rank)."""
    import subprocess
    import sys

    code = r'''
import os, torch, torch.nn.functional as F
import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.models import SimpleCNN
from distributeddataparallel_amd.utils.spawn import free_port
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(free_port())
pg = dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
torch.backends.cudnn.deterministic = True
torch.manual_seed(0)
model, ref = SimpleCNN().cuda(), SimpleCNN().cuda()
ddp = xddp.DDP(model, device_ids=[0], bucket_cap_mb=2)
opt = torch.optim.SGD(ddp.parameters(), lr=0.01)
for it in range(4):
    ref.load_state_dict(model.state_dict())
    x = torch.randn(16, 3, 32, 32, device="cuda"); y = torch.randint(0, 10, (16,), device="cuda")
    opt.zero_grad(); ref.zero_grad()
    F.cross_entropy(ddp(x), y).backward(); F.cross_entropy(ref(x), y).backward()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=0, atol=0)
    opt.step()
n = pg.comm.num_collectives()
recs = [r["op"] for r in pg.flight_records()]
assert recs.count("allreduce") >= 8, recs
t = torch.arange(6, device="cuda", dtype=torch.float32)
dist.all_reduce(t); dist.broadcast(t, 0); torch.cuda.synchronize()
assert torch.equal(t, torch.arange(6, device="cuda", dtype=torch.float32))
dist.destroy_process_group()
print("forced-launch ok", n)
'''
    env = dict(os.environ, XDDP_RCCL_FORCE_LAUNCH="1")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "forced-launch ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_rccl_forced_launch_debug_detail_grouped():
    """XDDP_DEBUG=DETAIL on the RCCL communicator with real RCCL kernels (W=1, forced launches):
    DDP iterations whose bucket bursts are RCCL groups (iteration 0's single launch, the rebuilt
    buckets' tail) and a nested coalescing() block run without a false desync and with exact
    gradients — the fingerprints go over the host helper ring, not through the open group. A
    wait() on a collective inside an open group raises instead of returning on a stale event."""
    import subprocess
    import sys

    code = r'''
import os, torch, pytest, torch.nn.functional as F
import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.models import SimpleCNN
from distributeddataparallel_amd.utils.spawn import free_port
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(free_port())
pg = dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
torch.backends.cudnn.deterministic = True
torch.manual_seed(0)
model, ref = SimpleCNN().cuda(), SimpleCNN().cuda()
ddp = xddp.DDP(model, device_ids=[0], bucket_cap_mb=1)
opt = torch.optim.SGD(ddp.parameters(), lr=0.01)
for it in range(4):
    ref.load_state_dict(model.state_dict())
    x = torch.randn(16, 3, 32, 32, device="cuda"); y = torch.randint(0, 10, (16,), device="cuda")
    opt.zero_grad(); ref.zero_grad()
    F.cross_entropy(ddp(x), y).backward(); F.cross_entropy(ref(x), y).backward()
    for p, q in zip(model.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad, rtol=0, atol=0)
    opt.step()
print("grouped launches", ddp._get_ddp_logging_data()["num_grouped_launches"])
a = torch.arange(6, device="cuda", dtype=torch.float32); b = torch.ones(1000, device="cuda", dtype=torch.bfloat16)
with dist.coalescing():
    dist.all_reduce(a)
    with dist.coalescing():
        w = dist.all_reduce(b, async_op=True)
        with pytest.raises(RuntimeError, match="inside an open group"):
            w.wait()
    dist.broadcast(a, 0)
w.wait(); torch.cuda.synchronize()
assert torch.equal(a, torch.arange(6, device="cuda", dtype=torch.float32)) and torch.equal(b, torch.ones_like(b))
recs = [r["op"] for r in pg.flight_records()]
assert recs.count("allreduce") >= 8, recs
dist.destroy_process_group()
print("detail ok")
'''
    env = dict(os.environ, XDDP_RCCL_FORCE_LAUNCH="1", XDDP_DEBUG="DETAIL")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "detail ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("schedule,grad_as_view", [("tail", False), ("tail", True), ("backward", False)])
def test_rccl_forced_launch_overlapped_optimizer(schedule, grad_as_view):
    """W=1 with real RCCL kernels on the comm stream (XDDP_RCCL_FORCE_LAUNCH=1): the overlapped
    optimizer (deferred updates under a chunked tail all-reduce, or per-bucket updates during
    backward) trains bitwise like backward-then-step, and .grad holds the reduced gradient after
    backward also without bucket views (the hook hands the reducer a completed future while the
    collectives are still in flight)."""
    import subprocess
    import sys

    code = r'''
import os, sys, torch, torch.nn.functional as F
import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.models.llama import llama_tiny
from distributeddataparallel_amd.optim import FusedAdamW
from distributeddataparallel_amd.utils.spawn import free_port
schedule, view = sys.argv[1], sys.argv[2] == "1"
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(free_port())
pg = dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
def make():  # a 2048 x 64 token embedding: the tail bucket is >= 4 chunks of 64 KB
    torch.manual_seed(0)
    return llama_tiny(max_seq_len=64, vocab_size=2048).cuda().to(torch.bfloat16)
m1, m2 = make(), make()
d1 = xddp.DDP(m1, device_ids=[0], gradient_as_bucket_view=view, bucket_cap_mb=0.25)
d2 = xddp.DDP(m2, device_ids=[0], gradient_as_bucket_view=view, bucket_cap_mb=0.25)
o1 = FusedAdamW(m1.parameters(), lr=1e-3, weight_decay=0.1, master_weights=True)
o2 = FusedAdamW(m2.parameters(), lr=1e-3, weight_decay=0.1, master_weights=True)
d1.register_overlapped_optimizer(o1, schedule=schedule, tail_chunk_bytes=1 << 16)
vocab = m1.tok_embeddings.weight.shape[0] if hasattr(m1, "tok_embeddings") else 256
g = torch.Generator(device="cuda").manual_seed(1)
for it in range(3):
    x = torch.randint(0, vocab, (2, 64), device="cuda", generator=g)
    y = torch.randint(0, vocab, (2, 64), device="cuda", generator=g)
    o1.zero_grad(set_to_none=False); o2.zero_grad(set_to_none=False)
    out = d1(x); F.cross_entropy(out.float().view(-1, out.shape[-1]), y.view(-1)).backward()
    out = d2(x); F.cross_entropy(out.float().view(-1, out.shape[-1]), y.view(-1)).backward()
    for a, b in zip(m1.parameters(), m2.parameters()):
        assert torch.equal(a.grad, b.grad), it
    o2.step()
torch.cuda.synchronize()
for a, b in zip(m1.parameters(), m2.parameters()):
    assert torch.equal(a, b)
if schedule == "tail":
    assert d1._overlap_state["last_chunks"] >= 2, d1._overlap_state["last_chunks"]
n = pg.comm.num_collectives()
dist.destroy_process_group()
print("overlap forced-launch ok", n)
'''
    env = dict(os.environ, XDDP_RCCL_FORCE_LAUNCH="1")
    r = subprocess.run([sys.executable, "-c", code, schedule, "1" if grad_as_view else "0"], env=env,
                       capture_output=True, text=True, timeout=240,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0 and "overlap forced-launch ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


@pytest.mark.parametrize("grad_as_view,accum", [(True, 1), (False, 2)])
def test_two_ranks_one_gpu_ddp_parity_peer_backend(grad_as_view, accum, monkeypatch):
    """The same W=2 DDP parity on the RCCL-free peer-memory backend: bucket all-reduces, the
    parameter/buffer broadcasts and the verification all-gather run as device-side one-shot
    kernels between the two processes (csrc/comm/peer_comm.cpp); a 1 MiB staging capacity makes the
    larger buckets take the chunked path."""
    monkeypatch.setenv("XDDP_PEER_CAPACITY_MB", "1")
    run_ranks(_w_gpu_parity, world=2, backend="peer", args=(grad_as_view, accum))


def _w_peer_collectives(rank, world):
    from distributeddataparallel_amd import distributed as dist

    torch.cuda.set_device(0)
    n = 300_001  # > the 64 KiB capacity set below: several chunks, ragged tail
    base = torch.arange(n, device="cuda", dtype=torch.float32)
    t = base + rank
    dist.all_reduce(t)
    torch.testing.assert_close(t, 2 * base + 1)
    t = base * (rank + 1)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    torch.testing.assert_close(t, base * world)
    t = (base + rank).to(torch.bfloat16)
    dist.all_reduce(t, op=dist.ReduceOp.AVG)
    torch.testing.assert_close(t.float(), (base + 0.5).to(torch.bfloat16).float(), rtol=1e-2, atol=1.0)
    t = torch.full((n,), float(rank), device="cuda")
    dist.broadcast(t, 1)
    assert torch.equal(t, torch.ones(n, device="cuda"))
    g = torch.empty(world * n, device="cuda")
    dist.all_gather_into_tensor(g, base + 10 * rank)
    assert torch.equal(g.view(world, n)[1], base + 10)
    out = torch.empty(n, device="cuda")
    dist.reduce_scatter_tensor(out, torch.cat([base, base + 1]) + rank)
    torch.testing.assert_close(out, 2 * (base + rank) + 1)
    dist.barrier()
    torch.cuda.synchronize()


def test_peer_backend_collectives(monkeypatch):
    """init_process_group("peer"): all-reduce (SUM / MAX / AVG in bf16), broadcast from rank 1,
    all-gather and reduce-scatter, all through the chunked path (64 KiB staging)."""
    monkeypatch.setenv("XDDP_PEER_CAPACITY_MB", "0.0625")
    run_ranks(_w_peer_collectives, world=2, backend="peer")
