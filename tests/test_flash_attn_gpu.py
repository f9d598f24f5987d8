"""Flash attention HIP kernels (csrc/kernels/flash_attn.hip) vs an fp32 PyTorch reference of the
same math: forward output, softmax LSE, and dq/dk/dv — at the ViT-L/16 head shape (D 64, 197 tokens,
non-causal), the Llama-3 shape (D 128, causal, GQA 4:1), and ragged edge cases."""
import math

import pytest
import torch

from distributeddataparallel_amd.ops.attention import flash_attention

pytestmark = pytest.mark.gpu


def _ref(q, k, v, causal, scale):
    B, S, H, D = q.shape
    Hkv = k.shape[2]
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if Hkv != H:
        kf = kf.repeat_interleave(H // Hkv, dim=1)
        vf = vf.repeat_interleave(H // Hkv, dim=1)
    s = qf @ kf.transpose(-1, -2) * scale
    if causal:
        m = torch.ones(S, k.shape[1], device=q.device, dtype=torch.bool).tril()
        s = s.masked_fill(~m, float("-inf"))
    p = s.softmax(-1)
    return (p @ vf).transpose(1, 2)


@pytest.mark.parametrize("B,S,H,Hkv,D,causal", [
    (2, 197, 16, 16, 64, False),    # ViT-L/16 head shape (ragged S)
    (16, 197, 16, 16, 64, False),   # ViT at a full-chip grid: the 8-wave whole-K/V forward
    (1, 512, 8, 2, 128, True),      # Llama-style causal GQA
    (2, 130, 4, 4, 128, True),      # ragged causal
    (1, 64, 2, 1, 64, True),        # one tile
    (3, 300, 2, 2, 128, False),     # ragged non-causal, D 128
    (2, 256, 4, 4, 64, False),      # one full 256-key dK/dV block (KW = 8 path)
    (3, 33, 2, 2, 64, False),       # short: most of the 256-key block masked
    (1, 100, 8, 2, 64, False),      # GQA on the one-block path
    (1, 257, 2, 2, 64, False),      # just past one block: two 128-key blocks
])
def test_flash_attention_matches_reference(B, S, H, Hkv, D, causal):
    torch.manual_seed(0)
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    scale = 1.0 / math.sqrt(D)
    o = flash_attention(q, k, v, causal=causal)
    qr, kr, vr = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _ref(qr, kr, vr, causal, scale)
    assert o.shape == (B, S, H, D) and o.dtype == torch.bfloat16
    torch.testing.assert_close(o.float(), ref, rtol=2e-2, atol=2e-2)
    g = torch.randn_like(ref)
    o.backward(g.to(torch.bfloat16))
    ref.backward(g.to(torch.bfloat16).float())
    for name, a, b in (("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad), ("dv", v.grad, vr.grad)):
        rel = ((a.float() - b).norm() / b.norm()).item()
        assert rel < 2e-2, (name, rel)


def test_flash_attention_strided_views():
    """q/k/v as strided views of one fused projection (ViT's qkv layout) give the same result."""
    torch.manual_seed(1)
    B, S, H, D = 2, 197, 4, 64
    qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16)
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o = flash_attention(q, k, v)
    o2 = flash_attention(q.contiguous(), k.contiguous(), v.contiguous())
    torch.testing.assert_close(o, o2, rtol=0, atol=0)
