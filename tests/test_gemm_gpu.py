"""Own transformer GEMM (csrc/kernels/gemm.hip: y = a · wᵀ on the LDS-DMA MFMA pipeline) against
an fp32 torch reference of the same op: plain, + bias, + bias -> GELU (pre-activation and
activation), + residual (in place, the pre-norm block's x += o · Woᵀ); M tails (rows past M
re-read row M - 1 and are not stored), both tile widths (N % 256 and N % 128 only), even and odd
K-tile counts (an odd count runs behind a zero tile)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _C():
    from distributeddataparallel_amd._native import load

    return load()


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


@pytest.mark.parametrize("M,K,N", [(1, 64, 128), (100, 128, 256), (300, 192, 384), (513, 1024, 1024),
                                   (12608 // 4, 1024, 3072), (2048, 4096, 1024)])
def test_gemm_nt_plain_and_bias(M, K, N):
    C = _C()
    g = torch.Generator(device="cuda").manual_seed(M + N)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    ref = a.float() @ w.float().t()
    y = C.gemm_nt(a, w)[0]
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    assert _rel(y, ref) < 5e-3
    yb = C.gemm_nt(a, w, b, 1)[0]
    assert _rel(yb, ref + b.float()) < 5e-3


@pytest.mark.parametrize("M,N,K", [(777, 1152, 512),    # N % 256 != 0: 256 x 128 tiles
                                   (777, 1024, 576),    # few tiles: 256 x 128 fills the CUs better
                                   (16384, 1024, 512)])  # 256 x 256 tiles (gemm.hip pick_bn)
def test_gemm_nt_gelu_and_residual(M, N, K):
    C = _C()
    g = torch.Generator(device="cuda").manual_seed(7)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    h, act = C.gemm_nt(a, w, b, 2)
    href = a.float() @ w.float().t() + b.float()
    assert _rel(h, href) < 5e-3
    # the activation is GELU of the stored (bf16) pre-activation
    assert _rel(act, F.gelu(h.float())) < 5e-3
    # residual: in place into x (x is the residual and the output), with and without a bias
    x = torch.randn(M, N, device="cuda", generator=g).to(torch.bfloat16)
    for bias in (None, b):
        xr = x.float() + a.float() @ w.float().t() + (0 if bias is None else bias.float())
        xx = x.clone()
        out = C.gemm_nt(a, w, bias, 3, xx, xx)[0]
        assert out.data_ptr() == xx.data_ptr()
        assert _rel(xx, xr) < 5e-3


def test_gemm_nt_rejects_bad_shapes():
    C = _C()
    a = torch.zeros(8, 100, device="cuda", dtype=torch.bfloat16)
    w = torch.zeros(128, 100, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError, match="K % 64"):
        C.gemm_nt(a, w)


def test_own_linear_autograd_matches_fp32(monkeypatch):
    """ops/linear.py with XDDP_OWN_GEMM=1: forward on gemm_nt (with the residual epilogue),
    backward on hipBLASLt."""
    from distributeddataparallel_amd.ops.linear import linear, own_gemm_ok

    monkeypatch.setenv("XDDP_OWN_GEMM", "1")

    g = torch.Generator(device="cuda").manual_seed(3)
    x = torch.randn(2, 200, 512, device="cuda", generator=g).to(torch.bfloat16).requires_grad_(True)
    w = (torch.randn(768, 512, device="cuda", generator=g) * 512 ** -0.5).to(torch.bfloat16).requires_grad_(True)
    r = torch.randn(2, 200, 768, device="cuda", generator=g).to(torch.bfloat16).requires_grad_(True)
    assert own_gemm_ok(x, w)
    y = linear(x, w, r)
    assert y.grad_fn is not None and "_Linear" in type(y.grad_fn).__name__
    dy = torch.randn_like(y)
    y.backward(dy)
    xf, wf, rf = (t.detach().float().requires_grad_(True) for t in (x, w, r))
    yf = rf + xf @ wf.t()
    yf.backward(dy.float())
    assert _rel(y, yf) < 5e-3
    for a, b in ((x.grad, xf.grad), (w.grad, wf.grad), (r.grad, rf.grad)):
        assert _rel(a, b) < 1e-2



@pytest.mark.parametrize("M,K,N", [(777, 512, 1024), (12608 // 8, 1024, 4096), (300, 192, 384)])
def test_gemm_nt_dgelu_bias_grad(M, K, N):
    """Epilogue 4 (the MLP's GELU backward in fc2's input-gradient GEMM): dh = (g·Wᵀ)·gelu'(h)
    and its column sums (fc1's bias gradient), vs fp32 torch autograd of GELU."""
    C = _C()
    g = torch.Generator(device="cuda").manual_seed(M)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    h = (torch.randn(M, N, device="cuda", generator=g) * 2).to(torch.bfloat16)
    b = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    dh, db = C.gemm_nt(a, w, b, 4, h)
    assert dh.shape == (M, N) and db.shape == (N,) and db.dtype == torch.bfloat16
    hf = h.float().requires_grad_()
    up = a.float() @ w.float().t()
    F.gelu(hf).backward(up)
    assert _rel(dh, hf.grad) < 1e-2
    assert _rel(db, hf.grad.sum(0)) < 1e-2
    _, db32 = C.gemm_nt(a, w, None, 4, h)  # no bias: fp32 sums
    assert db32.dtype == torch.float32 and _rel(db32, hf.grad.sum(0)) < 5e-3


@pytest.mark.parametrize("M,K,N,off", [(50176 // 8, 1024, 256, 0.0), (777, 2048, 512, 20.0), (300, 192, 384, 0.0)])
def test_gemm_nt_statistics_epilogue(M, K, N, off):
    """Epilogue 5: y = a @ w.T plus per-column BatchNorm statistics partials (group-minor
    [3, N, mtiles]) of the stored bf16 y — the deep-K 1x1 conv forward with its BN's statistics."""
    from distributeddataparallel_amd import native

    C = native()
    torch.manual_seed(3)
    a = (torch.randn(M, K, device="cuda") + off).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    y, part = C.gemm_nt(a, w, None, 5)
    ref = a.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    assert part.shape == (3, N, (M + 255) // 256)
    yf = y.float()
    rm, rv = torch.zeros(N, device="cuda"), torch.ones(N, device="cuda")
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    mean, invstd, _ = C.bn_stats_from_partials(part, M, None, None, rm, rv, nbt, 0.1, False, 1e-5, True)
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-5, atol=1e-4 * yf.std(0).max().item())
    torch.testing.assert_close(1.0 / invstd ** 2 - 1e-5, yf.var(0, unbiased=False), rtol=2e-3, atol=1e-6)
