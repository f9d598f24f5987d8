"""DDP on one MI355X through the RCCL communicator (W=1): the full native path runs —
store, RCCL comm, Reducer hooks, multi-tensor bucket kernels, fused optimizer."""
import os

import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.models import SimpleCNN
from distributeddataparallel_amd.utils.spawn import free_port

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg():
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    g = dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
    yield g
    dist.destroy_process_group()


def test_rccl_collectives_w1(pg):
    t = torch.arange(10, device="cuda", dtype=torch.float32)
    dist.all_reduce(t)
    torch.testing.assert_close(t, torch.arange(10, device="cuda", dtype=torch.float32))
    dist.all_reduce(t, op=dist.ReduceOp.AVG)
    dist.broadcast(t, 0)
    out = torch.empty(10, device="cuda")
    dist.all_gather_into_tensor(out, t)
    torch.testing.assert_close(out, t)
    dist.barrier()
    assert pg.comm.num_collectives() >= 5
    recs = pg.flight_records()
    assert recs[-1]["op"] == "barrier"


@pytest.mark.parametrize("grad_as_view", [False, True])
@pytest.mark.parametrize("comm_dtype", [None, torch.bfloat16])
def test_ddp_matches_local_training(pg, grad_as_view, comm_dtype):
    """W=1 DDP grads == plain-model grads (deterministic MIOpen; ref re-synced every step so
    only the reducer's own numerics are measured: exact for fp32, bf16 rounding otherwise)."""
    torch.backends.cudnn.deterministic = True
    try:
        torch.manual_seed(0)
        model = SimpleCNN().cuda()
        ref = SimpleCNN().cuda()
        ddp = xddp.DDP(model, device_ids=[0], gradient_as_bucket_view=grad_as_view, comm_dtype=comm_dtype)
        opt = torch.optim.SGD(ddp.parameters(), lr=0.01)
        for it in range(4):
            ref.load_state_dict(model.state_dict())
            x = torch.randn(16, 3, 32, 32, device="cuda")
            y = torch.randint(0, 10, (16,), device="cuda")
            opt.zero_grad()
            ref.zero_grad()
            F.cross_entropy(ddp(x), y).backward()
            F.cross_entropy(ref(x), y).backward()
            for (n, p), q in zip(model.named_parameters(), ref.parameters()):
                if comm_dtype is None:
                    torch.testing.assert_close(p.grad, q.grad, rtol=0, atol=0, msg=f"it{it} {n}")
                else:
                    scale = q.grad.abs().max().item() + 1e-12
                    assert (p.grad - q.grad).abs().max().item() <= 1e-2 * scale, (it, n)
            opt.step()
    finally:
        torch.backends.cudnn.deterministic = False
    assert ddp.reducer.native_launches() > 0, "native bucket kernels did not run"
    d = ddp._get_ddp_logging_data()
    assert d["has_rebuilt_buckets"] == "1"


@pytest.mark.parametrize("fused_bn", [False, True])
def test_ddp_bf16_channels_last_fused_sgd(pg, fused_bn):
    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d
    from distributeddataparallel_amd.optim import FusedSGD

    torch.manual_seed(0)
    m = resnet50(norm_layer=FusedBatchNorm2d if fused_bn else None).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    ddp = xddp.DDP(m, device_ids=[0], gradient_as_bucket_view=True)
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, master_weights=True)
    x = torch.randn(8, 3, 64, 64, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device="cuda")
    losses = []
    for _ in range(3):
        opt.zero_grad(set_to_none=True)
        loss = F.cross_entropy(ddp(x).float(), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    # grads alias bucket memory
    p0 = next(m.parameters())
    assert p0.grad is not None and p0.grad.data_ptr() != 0


def test_resnet50_fused_bn_matches_torch_bn(pg):
    """Same weights, same batch: fused-BN ResNet-50 forward/backward ≈ nn.BatchNorm2d ResNet-50 (fp32)."""
    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    torch.backends.cudnn.deterministic = True
    try:
        torch.manual_seed(0)
        a = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last)
        b = resnet50().cuda().to(memory_format=torch.channels_last)
        b.load_state_dict(a.state_dict())
        x = torch.randn(4, 3, 64, 64, device="cuda").contiguous(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (4,), device="cuda")
        la = F.cross_entropy(a(x), y)
        lb = F.cross_entropy(b(x), y)
        torch.testing.assert_close(la, lb, rtol=1e-3, atol=1e-3)
        la.backward()
        lb.backward()
        for (n, p), q in zip(a.named_parameters(), b.parameters()):
            # dγ = Σ dy·x̂ cancels heavily; summation-order differences show up at the 1e-2 level
            rel = ((p.grad - q.grad).norm() / (q.grad.norm() + 1e-12)).item()
            cos = F.cosine_similarity(p.grad.flatten(), q.grad.flatten(), dim=0).item()
            assert rel < 5e-2 and cos > 0.999, (n, rel, cos)
        for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
            torch.testing.assert_close(ba.float(), bb.float(), rtol=1e-3, atol=1e-4, msg=n)
    finally:
        torch.backends.cudnn.deterministic = False


def test_graphed_train_step_matches_eager():
    """Runs _graphed_train_step_check in a fresh process (MIOpen state such as solver choices and
    debug switches is per process; utils/graphs.py documents a replay NaN of MIOpen's Find-mode
    stem-conv solver that the capture's immediate mode avoids)."""
    import subprocess
    import sys

    code = ("import tests.test_ddp_gpu as t, os\n"
            "from distributeddataparallel_amd import distributed as dist\n"
            "from distributeddataparallel_amd.utils.spawn import free_port\n"
            "os.environ['MASTER_ADDR'] = '127.0.0.1'; os.environ['MASTER_PORT'] = str(free_port())\n"
            "dist.init_process_group('rccl', rank=0, world_size=1, device_id=0)\n"
            "t._graphed_train_step_check()\n"
            "dist.destroy_process_group()\n"
            "print('graphed ok')\n")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    r = subprocess.run([sys.executable, "-c", code], env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "graphed ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def _graphed_train_step_check():
    """HIP-graph capture of the whole DDP step (fwd, bwd + bucket all-reduce, FusedSGD): every
    replayed step equals an eager step taken from the same state (the eager model is re-synced
    from the graphed one before each step, in place, so MIOpen's run-to-run nondeterminism does
    not compound across steps)."""
    from distributeddataparallel_amd.ops import FusedBatchNorm2d
    from distributeddataparallel_amd.optim import FusedSGD
    from distributeddataparallel_amd.utils.graphs import GraphedTrainStep

    def make():
        torch.manual_seed(0)
        m = SimpleCNN(norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last)
        d = xddp.DDP(m, device_ids=[0], gradient_as_bucket_view=True)
        return m, d, FusedSGD(d.parameters(), lr=0.05, momentum=0.9)

    g = torch.Generator(device="cuda").manual_seed(3)
    xs = [torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
          for _ in range(6)]
    ys = [torch.randint(0, 10, (32,), device="cuda", generator=g) for _ in range(6)]
    lf = F.cross_entropy
    m2, d2, o2 = make()
    step = GraphedTrainStep(d2, o2, lf, xs[0], ys[0], warmup_steps=3)
    m3, d3, o3 = make()
    for _ in range(2):  # create momentum buffers / rebuild buckets on the eager side
        o3.zero_grad(set_to_none=True)
        lf(d3(xs[0]), ys[0]).backward()
        o3.step()
    for x, y in zip(xs, ys):
        p0 = [p.detach().clone() for p in m2.parameters()]
        with torch.no_grad():
            for a, b in zip(m2.parameters(), m3.parameters()):
                b.copy_(a)
                o3.state[b]["momentum_buffer"].copy_(o2.state[a]["momentum_buffer"])
            for a, b in zip(m2.buffers(), m3.buffers()):
                b.copy_(a)
        o3.zero_grad(set_to_none=True)
        loss3 = lf(d3(x), y)
        loss3.backward()
        o3.step()
        loss2 = step(x, y)
        torch.cuda.synchronize()
        torch.testing.assert_close(loss2, loss3, rtol=1e-3, atol=1e-4)
        # compare the step's updates (capture runs MIOpen in immediate mode, the eager model in
        # find mode, so the two use different conv algorithms; their fp32 reduction-order noise is
        # a relative error of the update — up to ~1 % on the small layer4 gradients — not of the
        # weight)
        for (n, a), b, q in zip(m2.named_parameters(), m3.parameters(), p0):
            u2, u3 = (a - q).flatten(), (b - q).flatten()
            err = float((u2 - u3).norm() / (u3.norm() + 1e-12))
            assert err < 3e-2, (n, err)
        for (n, a), b in zip(m2.named_buffers(), m3.buffers()):
            if a.is_floating_point():
                torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-5, msg=lambda m, n=n: f"{n}: {m}")
            else:
                assert torch.equal(a, b), n


@pytest.mark.parametrize("which", ["llama", "vit"])
def test_transformer_ddp_fused_norms_adamw(pg, which):
    """Transformer configs on the native path: fused LayerNorm/RMSNorm kernels, bucketed DDP,
    FusedAdamW with fp32 master weights (bf16 params) — grads match a plain model."""
    from distributeddataparallel_amd.models import llama_tiny, vit_tiny
    from distributeddataparallel_amd.optim import FusedAdamW

    def make():
        torch.manual_seed(0)
        return (llama_tiny() if which == "llama" else vit_tiny(num_classes=10)).cuda()

    m, ref = make(), make()
    ddp = xddp.DDP(m, device_ids=[0], bucket_cap_mb=0.05, first_bucket_cap_mb=0.01, gradient_as_bucket_view=True)
    if which == "llama":
        x = torch.randint(0, 512, (4, 32), device="cuda")
        y = torch.randint(0, 512, (4, 32), device="cuda")
        lf = lambda o, t: F.cross_entropy(o.float().reshape(-1, o.shape[-1]), t.reshape(-1))  # noqa: E731
    else:
        x = torch.randn(4, 3, 32, 32, device="cuda")
        y = torch.randint(0, 10, (4,), device="cuda")
        lf = lambda o, t: F.cross_entropy(o.float(), t)  # noqa: E731
    for _ in range(2):
        ref.load_state_dict(m.state_dict())
        m.zero_grad(set_to_none=True)
        ref.zero_grad(set_to_none=True)
        lf(ddp(x), y).backward()
        lf(ref(x), y).backward()
        for (n, a), b in zip(m.named_parameters(), ref.parameters()):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-5, msg=n)
    assert len(ddp.reducer.bucket_sizes_bytes()) > 1
    # bf16 model + fp32-master AdamW steps through the fused kernel
    mb = make().to(torch.bfloat16)
    ddpb = xddp.DDP(mb, device_ids=[0], gradient_as_bucket_view=True)
    opt = FusedAdamW(ddpb.parameters(), lr=1e-3, master_weights=True)
    losses = []
    for _ in range(5):
        opt.zero_grad(set_to_none=True)
        xx = x if which == "llama" else x.to(torch.bfloat16)
        loss = lf(ddpb(xx), y)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0], losses


def test_mixed_precision_and_delayed_allreduce_gpu(pg):
    """T6i/T6j on the RCCL path: bf16 param copies by one multi-tensor launch, fp32 grads; a
    delayed flat-buffer all-reduce for the stem params."""
    from types import SimpleNamespace

    from torch.func import functional_call

    from distributeddataparallel_amd.models import MLP

    torch.manual_seed(0)
    m, base = MLP(3 * 32 * 32, 256, 10).cuda(), MLP(3 * 32 * 32, 256, 10).cuda()
    base.load_state_dict(m.state_dict())
    named = list(m.named_parameters())
    mp = SimpleNamespace(param_dtype=torch.bfloat16, reduce_dtype=torch.bfloat16, buffer_dtype=None)
    ddp = xddp.DDP(m, device_ids=[0], mixed_precision=mp, delay_all_reduce_named_params=named[:2],
                   param_to_hook_all_reduce=named[0][1])
    x = torch.randn(8, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (8,), device="cuda")
    out = ddp(x)
    assert out.dtype == torch.bfloat16
    F.cross_entropy(out.float(), y).backward()
    casted = {n: p.to(torch.bfloat16) for n, p in base.named_parameters()}
    F.cross_entropy(functional_call(base, casted, (x.to(torch.bfloat16),)).float(), y).backward()
    for (n, a), b in zip(m.named_parameters(), base.parameters()):
        assert a.grad is not None and a.grad.dtype == torch.float32, n
        cos = F.cosine_similarity(a.grad.flatten(), b.grad.flatten(), dim=0)
        assert cos > 0.99, (n, float(cos))


def test_overlapped_optimizer_matches_step_after_backward(pg):
    """register_overlapped_optimizer on GPU: the per-bucket FusedAdamW steps run on a side HIP
    stream during backward; the trained bf16 model (with fp32 masters) is bitwise the
    backward-then-step one (stream ordering: the side stream waits for each bucket's gradients,
    the compute stream for the side stream at the end of backward)."""
    from distributeddataparallel_amd.models.llama import llama_tiny
    from distributeddataparallel_amd.optim import FusedAdamW

    def make():
        torch.manual_seed(0)
        return llama_tiny(max_seq_len=64).cuda().to(torch.bfloat16)

    m1, m2 = make(), make()
    d1 = xddp.DDP(m1, device_ids=[0], gradient_as_bucket_view=True, bucket_cap_mb=0.5)
    d2 = xddp.DDP(m2, device_ids=[0], gradient_as_bucket_view=True, bucket_cap_mb=0.5)
    o1 = FusedAdamW(m1.parameters(), lr=1e-3, weight_decay=0.1, master_weights=True)
    o2 = FusedAdamW(m2.parameters(), lr=1e-3, weight_decay=0.1, master_weights=True)
    d1.register_overlapped_optimizer(o1)
    vocab = m1.tok_embeddings.weight.shape[0] if hasattr(m1, "tok_embeddings") else 256
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(3):
        x = torch.randint(0, vocab, (2, 64), device="cuda", generator=g)
        y = torch.randint(0, vocab, (2, 64), device="cuda", generator=g)
        for d, o, overlapped in ((d1, o1, True), (d2, o2, False)):
            o.zero_grad(set_to_none=True)
            out = d(x)
            F.cross_entropy(out.float().view(-1, out.shape[-1]), y.view(-1)).backward()
            if not overlapped:
                o.step()
    torch.cuda.synchronize()
    for a, b in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, b, rtol=0, atol=0)


def test_grad_targets_write_weight_grads_into_buckets(pg):
    """With gradient_as_bucket_view, the linears of ops/linear.py write their weight gradients
    straight into the DDP bucket views (set_grad_targets): the gradients are bitwise those of the
    plain model, the weights' .grad ARE their bucket views after backward (no copy into the
    bucket), and a weight used twice in one forward still gets the sum of both uses."""
    import copy

    import torch.nn.functional as F

    from distributeddataparallel_amd.models.llama import llama_tiny
    from distributeddataparallel_amd.ops.linear import linear

    class Twice(nn.Module):  # one weight, two uses: only the first may take the target
        def __init__(self):
            super().__init__()
            self.lin = nn.Linear(64, 64, bias=False)

        def forward(self, x):
            return linear(linear(x, self.lin.weight), self.lin.weight, x).sum(1)

    torch.manual_seed(0)
    for make in (lambda: llama_tiny(max_seq_len=64).cuda().to(torch.bfloat16),
                 lambda: Twice().cuda().to(torch.bfloat16)):
        m = make()
        ref = copy.deepcopy(m)
        d = xddp.DDP(m, device_ids=[0], gradient_as_bucket_view=True, bucket_cap_mb=0.25)
        g = torch.Generator(device="cuda").manual_seed(1)
        for it in range(3):
            if isinstance(m, Twice):
                x = torch.randn(4, 16, 64, device="cuda", generator=g).to(torch.bfloat16)
                loss_of = lambda mod: mod(x).float().square().mean()  # noqa: E731
            else:
                x = torch.randint(0, 512, (2, 64), device="cuda", generator=g)
                loss_of = lambda mod: F.cross_entropy(mod(x).float().view(-1, 512), x.view(-1))  # noqa: E731
            for p in list(m.parameters()) + list(ref.parameters()):
                p.grad = None
            loss_of(d).backward()
            loss_of(ref).backward()
            for (n, a), b in zip(m.named_parameters(), ref.parameters()):
                assert (a.grad is None) == (b.grad is None), n
                if a.grad is not None:
                    assert torch.equal(a.grad, b.grad), (it, n)
            with torch.no_grad():
                for a, b in zip(m.parameters(), ref.parameters()):
                    if a.grad is not None:
                        a.sub_(0.01 * a.grad)
                        b.sub_(0.01 * b.grad)
        views = d.reducer.param_bucket_views()
        aliased = [n for (n, p), v in zip(m.named_parameters(), views)
                   if p.grad is not None and v is not None and p.grad.data_ptr() == v.data_ptr()]
        if not isinstance(m, Twice):
            assert any("wq" in n for n in aliased) and any("w2" in n for n in aliased), aliased
