"""HIP multi-tensor kernels vs plain PyTorch fp32 references (gfx950)."""
import pytest
import torch

from distributeddataparallel_amd._native import load
from distributeddataparallel_amd.optim import FusedAdamW, FusedSGD, clip_grad_norm_

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _shapes():
    return [(7,), (1000,), (64, 3, 7, 7), (513, 129), (8193,), (1,), (3, 5)]


@pytest.mark.parametrize("src_dt,dst_dt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                           (torch.bfloat16, torch.float32), (torch.bfloat16, torch.bfloat16),
                                           (torch.float16, torch.float32)])
def test_scale_copy(src_dt, dst_dt):
    C = load()
    src = [torch.randn(s, device=DEV).to(src_dt) for s in _shapes()]
    dst = [torch.empty(s, device=DEV, dtype=dst_dt) for s in _shapes()]
    C.mt_scale_copy(src, dst, 0.5)
    for a, b in zip(src, dst):
        torch.testing.assert_close(b.float(), (a.float() * 0.5).to(dst_dt).float(), rtol=1e-2 if dst_dt != torch.float32 else 1e-6, atol=1e-6)


def test_scale_copy_many_tensors_and_misaligned():
    C = load()
    base = torch.randn(100_003, device=DEV)
    src = [base[i * 997 + 1: i * 997 + 1 + 500] for i in range(90)]  # > one segment table, 4-B aligned only
    dst = [torch.empty(500, device=DEV) for _ in src]
    scale = torch.tensor([2.0], device=DEV)
    C.mt_scale_copy(src, dst, 1.5, scale)
    for a, b in zip(src, dst):
        torch.testing.assert_close(b, a * 3.0)


def test_channels_last_copy():
    C = load()
    a = torch.randn(8, 16, 5, 5, device=DEV).contiguous(memory_format=torch.channels_last)
    b = torch.empty_like(a)
    C.mt_scale_copy([a], [b], 1.0)
    torch.testing.assert_close(a, b)


def test_pack_unpack_roundtrip():
    C = load()
    ts = [torch.randn(s, device=DEV) for s in _shapes()]
    offs, o = [], 0
    for t in ts:
        offs.append(o)
        o = (o + t.numel() + 15) // 16 * 16
    flat = torch.zeros(o, device=DEV)
    C.mt_pack(ts, flat, offs)
    outs = [torch.empty_like(t) for t in ts]
    C.mt_unpack(flat, offs, outs)
    for a, b in zip(ts, outs):
        torch.testing.assert_close(a, b)


def test_copy_bytes_bit_exact_mixed_dtypes():
    C = load()
    g = torch.Generator(device=DEV).manual_seed(0)
    raw = torch.randint(-2**62, 2**62, (4097,), device=DEV, dtype=torch.int64, generator=g)
    src = [raw[:1], raw[1:9].view(torch.float64), raw[:100].view(torch.float32)[1:33],  # 4-B aligned only
           raw[:50].view(torch.bfloat16)[3:101], raw.view(torch.uint8)[5:20000],  # odd byte offsets
           torch.full((3,), float("nan"), device=DEV, dtype=torch.bfloat16)]
    dst = [torch.empty_like(t) for t in src]
    C.mt_copy_bytes(src, dst)
    for a, b in zip(src, dst):
        assert torch.equal(a.view(torch.uint8) if a.dtype != torch.uint8 else a,
                           b.view(torch.uint8) if b.dtype != torch.uint8 else b)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_l2norm_and_clip(dt):
    C = load()
    ts = [torch.randn(s, device=DEV).to(dt) for s in _shapes()]
    out = torch.empty(2, device=DEV)
    C.mt_l2norm(ts, out, 1.0)
    ref = torch.linalg.vector_norm(torch.cat([t.float().flatten() for t in ts]))
    torch.testing.assert_close(out[0], ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(out[1], torch.clamp(1.0 / (ref + 1e-6), max=1.0), rtol=1e-4, atol=1e-6)


def test_clip_grad_norm_matches_torch():
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in _shapes()]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    for p, q in zip(ps, qs):
        g = torch.randn_like(p) * 3
        p.grad, q.grad = g.clone(), g.clone()
    n1 = clip_grad_norm_(ps, 0.5)
    n2 = torch.nn.utils.clip_grad_norm_(qs, 0.5)
    torch.testing.assert_close(n1, n2, rtol=1e-5, atol=1e-5)
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-6)


def test_nonfinite():
    C = load()
    flag = torch.empty(1, dtype=torch.int32, device=DEV)
    ts = [torch.randn(100, device=DEV), torch.randn(10000, device=DEV)]
    C.mt_nonfinite(ts, flag)
    assert flag.item() == 0
    ts[1][777] = float("nan")
    C.mt_nonfinite(ts, flag)
    assert flag.item() == 1


@pytest.mark.parametrize("nesterov,wd,mom", [(False, 0.0, 0.0), (False, 1e-4, 0.9), (True, 1e-2, 0.9)])
def test_fused_sgd_matches_torch(nesterov, wd, mom):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in _shapes()]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    o1 = FusedSGD(ps, lr=0.1, momentum=mom, weight_decay=wd, nesterov=nesterov)
    o2 = torch.optim.SGD(qs, lr=0.1, momentum=mom, weight_decay=wd, nesterov=nesterov)
    for _ in range(3):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-6)


def test_fused_sgd_master_weights_bf16():
    torch.manual_seed(0)
    ref = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in _shapes()]
    ps = [torch.nn.Parameter(r.detach().to(torch.bfloat16)) for r in ref]
    refq = [torch.nn.Parameter(p.detach().float()) for p in ps]
    o1 = FusedSGD(ps, lr=0.05, momentum=0.9, weight_decay=1e-4, master_weights=True)
    o2 = torch.optim.SGD(refq, lr=0.05, momentum=0.9, weight_decay=1e-4)
    for _ in range(4):
        for p, q in zip(ps, refq):
            g = torch.randn(p.shape, device=DEV)
            p.grad, q.grad = g.to(torch.bfloat16), g.to(torch.bfloat16).float()
        o1.step()
        o2.step()
    for p, q in zip(ps, refq):
        torch.testing.assert_close(o1.state[p]["master"], q.detach(), rtol=1e-5, atol=1e-5)
        # the bf16 param is the rounded master: at most one bf16 ulp from the rounded reference
        torch.testing.assert_close(p.float(), o1.state[p]["master"].to(torch.bfloat16).float(), rtol=0, atol=0)
        torch.testing.assert_close(p.float(), q.detach().float(), rtol=8e-3, atol=1e-5)


@pytest.mark.parametrize("wd", [0.0, 0.01])
def test_fused_adamw_matches_torch(wd):
    torch.manual_seed(0)
    ps = [torch.nn.Parameter(torch.randn(s, device=DEV)) for s in _shapes()]
    qs = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    o1 = FusedAdamW(ps, lr=1e-2, weight_decay=wd)
    o2 = torch.optim.AdamW(qs, lr=1e-2, weight_decay=wd)
    for _ in range(5):
        for p, q in zip(ps, qs):
            g = torch.randn_like(p)
            p.grad, q.grad = g.clone(), g.clone()
        o1.step()
        o2.step()
    for p, q in zip(ps, qs):
        torch.testing.assert_close(p, q, rtol=1e-5, atol=1e-5)
