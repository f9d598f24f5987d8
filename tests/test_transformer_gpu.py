"""Fused RoPE / SwiGLU HIP kernels (csrc/kernels/transformer.hip) vs plain PyTorch fp32 references,
and the Llama block built on them."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _tables(S, Dh):
    from distributeddataparallel_amd.models.llama import _rope_table

    cos, sin = _rope_table(Dh, S + 5, 500000.0, device="cuda")
    return cos.contiguous(), sin.contiguous()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(2, 17, 4, 128), (1, 64, 8, 64), (3, 5, 2, 16)])
def test_rope_matches_reference(dt, shape):
    from distributeddataparallel_amd.ops.transformer import rope

    torch.manual_seed(0)
    B, S, H, Dh = shape
    cos, sin = _tables(S, Dh)
    x = torch.randn(shape, device="cuda").to(dt)
    x1 = x.clone().requires_grad_()
    x2 = x.float().clone().requires_grad_()
    y1 = rope(x1, cos, sin)
    c, s = cos[:S][None, :, None, :], sin[:S][None, :, None, :]
    a, b = x2[..., 0::2], x2[..., 1::2]
    y2 = torch.stack([a * c - b * s, a * s + b * c], dim=-1).flatten(-2)
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(y1.float(), y2, **tol)
    g = torch.randn(shape, device="cuda")
    y1.backward(g.to(dt))
    y2.backward(g.to(dt).float())
    torch.testing.assert_close(x1.grad.float(), x2.grad, **tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_swiglu_matches_reference(dt):
    from distributeddataparallel_amd.ops.transformer import swiglu

    torch.manual_seed(1)
    a = (torch.randn(37, 96, device="cuda") * 3).to(dt)
    b = torch.randn(37, 96, device="cuda").to(dt)
    a1, b1 = a.clone().requires_grad_(), b.clone().requires_grad_()
    a2, b2 = a.float().clone().requires_grad_(), b.float().clone().requires_grad_()
    h1 = swiglu(a1, b1)
    h2 = F.silu(a2) * b2
    tol = dict(rtol=1e-5, atol=1e-5) if dt == torch.float32 else dict(rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(h1.float(), h2, **tol)
    g = torch.randn_like(h2)
    h1.backward(g.to(dt))
    h2.backward(g.to(dt).float())
    torch.testing.assert_close(a1.grad.float(), a2.grad, **tol)
    torch.testing.assert_close(b1.grad.float(), b2.grad, **tol)


def test_llama_block_fused_matches_reference_ops(monkeypatch):
    """llama_tiny with the fused kernels vs the same weights on the PyTorch reference ops."""
    from distributeddataparallel_amd.models import llama_tiny

    torch.manual_seed(2)
    m = llama_tiny().cuda()
    x = torch.randint(0, 512, (2, 64), device="cuda")
    outs, grads = [], []
    for flag in ("1", "0"):
        monkeypatch.setenv("XDDP_FUSED_TRANSFORMER", flag)
        m.zero_grad()
        o = m(x)
        o.float().pow(2).mean().backward()
        outs.append(o.detach().float())
        grads.append(torch.cat([p.grad.flatten() for p in m.parameters()]))
    torch.testing.assert_close(outs[0], outs[1], rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(grads[0], grads[1], rtol=1e-3, atol=1e-6)
