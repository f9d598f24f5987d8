"""Fused transformer encoder block (ops/encoder_block.py) and its kernels vs fp32 PyTorch.

Each fused kernel is checked against a plain fp32 PyTorch computation of the same op; the whole
block is checked against an fp32 copy of the module (torch ops + SDPA), with the unfused bf16
module path as the yardstick for the error a bf16 stack is allowed.
"""
import copy
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

from distributeddataparallel_amd._native import load  # noqa: E402
from distributeddataparallel_amd.models.vit import EncoderBlock  # noqa: E402
from distributeddataparallel_amd.ops.encoder_block import encoder_block_supported  # noqa: E402
from distributeddataparallel_amd.ops.layer_norm import FusedLayerNorm  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def test_ln_forward_add_bias_and_residual_backward():
    C = load()
    torch.manual_seed(0)
    rows, D = 1000, 1024
    x = torch.randn(rows, D, device="cuda").bfloat16()
    w = (1 + 0.1 * torch.randn(D, device="cuda")).bfloat16()
    b = (0.1 * torch.randn(D, device="cuda")).bfloat16()
    ab = torch.randn(D, device="cuda").bfloat16()
    y, mean, rstd, xb = C.ln_forward(x, w, b, 1e-6, False, ab)
    ref = F.layer_norm(x.float(), (D,), w.float(), b.float(), 1e-6)
    assert rel(y, ref) < 5e-3
    assert torch.equal(xb, (x.float() + ab.float()).bfloat16())
    dy = torch.randn(rows, D, device="cuda").bfloat16()
    res = torch.randn(rows, D, device="cuda").bfloat16()
    dx, dw, db, sres, sout = C.ln_backward(dy, x, w, mean, rstd, False, True, True, res)
    xf = x.float().requires_grad_()
    wf, bf = w.float().requires_grad_(), b.float().requires_grad_()
    F.layer_norm(xf, (D,), wf, bf, 1e-6).backward(dy.float())
    dx_ref = xf.grad + res.float()
    assert rel(dx, dx_ref) < 5e-3
    assert rel(dw, wf.grad) < 5e-3 and rel(db, bf.grad) < 5e-3
    assert rel(sres, res.float().sum(0)) < 5e-3
    assert rel(sout, dx_ref.sum(0)) < 5e-3


@pytest.mark.parametrize("N", [1024, 3072, 4096])
def test_bias_grad_and_gelu_backward(N):
    C = load()
    torch.manual_seed(1)
    rows = 3001
    g = torch.randn(rows, N, device="cuda").bfloat16()
    h = (2 * torch.randn(rows, N, device="cuda")).bfloat16()
    bias = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    db, none = C.bias_grad(g, None, bias)
    assert none is None or not none.numel()
    assert rel(db, g.float().sum(0)) < 5e-3
    db1, dh = C.bias_grad(g, h, bias)
    hf = h.float().requires_grad_()
    F.gelu(hf).backward(g.float())
    assert rel(dh, hf.grad) < 5e-3
    assert rel(db1, hf.grad.sum(0)) < 5e-3
    a = C.gelu_forward(h)
    assert rel(a, F.gelu(h.float())) < 5e-3


def test_flash_backward_into_packed_gradient():
    C = load()
    torch.manual_seed(2)
    B, S, H, Dh = 2, 197, 16, 64
    qkv = torch.randn(B, S, 3, H, Dh, device="cuda").bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = C.flash_attn_forward(q, k, v, False, Dh ** -0.5)
    do = torch.randn(B, S, H, Dh, device="cuda").bfloat16()
    dq, dk, dv = C.flash_attn_backward(do, q, k, v, o, lse, False, Dh ** -0.5)
    d = torch.empty_like(qkv)
    C.flash_attn_backward(do, q, k, v, o, lse, False, Dh ** -0.5, d[:, :, 0], d[:, :, 1], d[:, :, 2])
    assert torch.equal(d[:, :, 0], dq) and torch.equal(d[:, :, 1], dk) and torch.equal(d[:, :, 2], dv)


@pytest.mark.parametrize("bias_dtype", [torch.bfloat16, torch.float32])
def test_flash_backward_qkv_bias_gradient(bias_dtype):
    """The one-block kernel's qkv bias gradient ([3][H][D]) against float sums of the bf16 dQ, dK, dV
    it wrote: Σ dQ from its dQ tiles, Σ dV as Σ dO (softmax rows sum to 1), Σ dK exactly 0 (Σ_k dS = 0;
    the summed bf16 dK is rounding noise, small against |dK|); dQ, dK, dV themselves are unchanged."""
    C = load()
    torch.manual_seed(3)
    B, S, H, Dh = 3, 197, 16, 64
    qkv = torch.randn(B, S, 3, H, Dh, device="cuda").bfloat16()
    q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
    o, lse = C.flash_attn_forward(q, k, v, False, Dh ** -0.5)
    do = torch.randn(B, S, H, Dh, device="cuda").bfloat16()
    d = torch.empty_like(qkv)
    bias = torch.zeros(3 * H * Dh, device="cuda", dtype=bias_dtype)
    res = C.flash_attn_backward(do, q, k, v, o, lse, False, Dh ** -0.5, d[:, :, 0], d[:, :, 1], d[:, :, 2], bias)
    assert len(res) == 4 and res[3] is not None and res[3].dtype == bias_dtype and res[3].shape == (3 * H * Dh,)
    ref = d.float().sum((0, 1))  # [3, H, Dh]
    got = res[3].float().view(3, H, Dh)
    for t in (0, 2):
        assert ((got[t] - ref[t]).norm() / ref[t].norm()).item() < 1e-2, t
    assert torch.count_nonzero(got[1]) == 0
    assert ref[1].norm() < 1e-2 * d[:, :, 1].float().abs().sum((0, 1)).norm()
    dq, dk, dv = C.flash_attn_backward(do, q, k, v, o, lse, False, Dh ** -0.5)
    assert torch.equal(d[:, :, 0], dq) and torch.equal(d[:, :, 1], dk) and torch.equal(d[:, :, 2], dv)
    # a path the fused sums do not cover (causal): the 4th output is None
    res = C.flash_attn_backward(do, q, k, v, o, lse, True, Dh ** -0.5, None, None, None, bias)
    assert len(res) == 4 and res[3] is None


def _run(blk, x, gout, fused_env):
    old = os.environ.get("XDDP_FUSED_BLOCK")
    os.environ["XDDP_FUSED_BLOCK"] = fused_env
    try:
        blk.zero_grad(set_to_none=True)
        xi = x.detach().clone().requires_grad_()
        out = blk(xi)
        out.backward(gout)
        grads = {n: p.grad.detach().clone() for n, p in blk.named_parameters()}
        return out.detach(), xi.grad.detach(), grads
    finally:
        if old is None:
            os.environ.pop("XDDP_FUSED_BLOCK", None)
        else:
            os.environ["XDDP_FUSED_BLOCK"] = old


@pytest.mark.parametrize("own", ["0", "bwd", "1"])
def test_fused_encoder_block_matches_fp32(own, monkeypatch):
    """The fused block on hipBLASLt only (0), with fc2's dgrad + dGELU + bias-gradient on the own
    GEMM (bwd, default), and with every projection on the own GEMM (1)."""
    monkeypatch.setenv("XDDP_OWN_GEMM", own)
    torch.manual_seed(3)
    D, H, MLP = 1024, 16, 4096
    blk32 = EncoderBlock(D, H, MLP, FusedLayerNorm).cuda()
    for p in blk32.parameters():  # non-trivial LN affine and biases so every gradient is exercised
        with torch.no_grad():
            p.add_(0.05 * torch.randn_like(p))
    blk16 = copy.deepcopy(blk32).bfloat16()
    x = torch.randn(4, 197, D, device="cuda")
    gout = torch.randn(4, 197, D, device="cuda")
    assert encoder_block_supported(x.bfloat16(), blk16)
    o32, dx32, g32 = _run(blk32, x, gout, "1")
    of, dxf, gf = _run(blk16, x.bfloat16(), gout.bfloat16(), "1")
    ou, dxu, gu = _run(blk16, x.bfloat16(), gout.bfloat16(), "0")
    # bf16 storage of every activation bounds both stacks at ~1e-2 relative; the fused path must
    # not be noticeably worse than the unfused bf16 module (same kernels minus the fusions)
    errs = {"out": (rel(of, o32), rel(ou, o32)), "dx": (rel(dxf, dx32), rel(dxu, dx32))}
    for n in g32:
        errs[n] = (rel(gf[n], g32[n]), rel(gu[n], g32[n]))
    for n, (ef, eu) in errs.items():
        assert ef < 3e-2, (n, ef, eu)
        assert ef <= 1.5 * eu + 3e-3, (n, ef, eu)


@pytest.mark.parametrize("R,Cc", [(1024, 4096), (77, 130), (1, 64), (192, 136)])
def test_transpose16_matches_torch(R, Cc):
    """The LDS-tiled 16-bit transpose (transformer.hip) equals torch's .t().contiguous() exactly."""
    from distributeddataparallel_amd import native

    x = torch.randn(R, Cc, device="cuda").to(torch.bfloat16)
    assert torch.equal(native().transpose16(x), x.t().contiguous())
