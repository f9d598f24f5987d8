"""1x1-conv MFMA GEMM with fused BatchNorm prologue/epilogue (csrc/kernels/conv_gemm.hip) vs
plain PyTorch fp32 references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

from distributeddataparallel_amd._native import load

pytestmark = pytest.mark.gpu

C = load() if torch.cuda.is_available() else None


def _x(b, c, h, w, offset=0.0):
    x = torch.randn(b, c, h, w, device="cuda") + offset
    return x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("b,cin,h,w,cout,s", [
    (2, 64, 14, 14, 256, 1),    # M = 392: partial last M-tile
    (3, 128, 9, 7, 64, 1),      # N = 64 tile variant, odd spatial size
    (2, 256, 15, 15, 512, 2),   # strided (downsample) row mapping, odd input size
    (1, 1024, 7, 7, 128, 1),    # long K loop (16 K-tiles)
])
def test_conv1x1_gemm_matches_conv2d(b, cin, h, w, cout, s):
    torch.manual_seed(0)
    x = _x(b, cin, h, w)
    wt = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
    y, part = C.conv1x1_gemm(x, wt, s, None, True)
    ref = F.conv2d(x.float(), wt.float(), stride=s)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    # prologue: relu(x * scale + shift) per input channel, applied before the product
    ss = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda")]).contiguous()
    yp, _ = C.conv1x1_gemm(x, wt, s, ss, False)
    xp = torch.relu(x.float() * ss[0].view(1, -1, 1, 1) + ss[1].view(1, -1, 1, 1)).to(torch.bfloat16).float()
    refp = F.conv2d(xp, wt.float(), stride=s)
    torch.testing.assert_close(yp.float(), refp, rtol=1e-2, atol=1e-2 * refp.abs().max().item())


@pytest.mark.parametrize("b,cin,h,w,cout,s,wdt", [
    (2, 64, 14, 14, 256, 1, torch.bfloat16),    # M = 392: partial last pixel step
    (3, 128, 9, 7, 64, 1, torch.float32),       # 64-wide tiles, fp32 weight output
    (2, 256, 15, 15, 512, 2, torch.bfloat16),   # strided (downsample) rows, odd input size
    (8, 64, 28, 28, 64, 1, torch.bfloat16),     # one tile, many M slabs (reduce split)
])
def test_conv1x1_wgrad_matches_fp32(b, cin, h, w, cout, s, wdt):
    """dW[n, k] = sum_m dY[m, n] X[m, k] (strided pixel rows for s = 2) against fp32 torch."""
    torch.manual_seed(2)
    x = _x(b, cin, h, w)
    oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
    dy = _x(b, cout, oh, ow)
    like = torch.empty(cout, cin, 1, 1, device="cuda", dtype=wdt)
    dw = C.conv1x1_wgrad(dy, x, s, like)
    xs = x.float()[:, :, ::s, ::s]
    ref = torch.einsum("bnhw,bkhw->nk", dy.float(), xs).view(cout, cin, 1, 1)
    assert dw.shape == ref.shape and dw.dtype == wdt
    tol = 1e-2 if wdt == torch.bfloat16 else 1e-4
    torch.testing.assert_close(dw.float(), ref, rtol=tol, atol=tol * ref.abs().max().item())


@pytest.mark.parametrize("b,cin,h,w,cout,s,pro", [
    (4, 256, 14, 14, 1024, 1, 0),   # layer-3 conv3 shape class, M = 784: 12.25 pixel steps per range
    (2, 512, 7, 7, 2048, 1, 0),     # 64 tiles, one pixel step per slice
    (3, 1024, 13, 13, 512, 2, 0),   # strided rows (downsample), odd input size
    (5, 128, 11, 9, 256, 1, 2),     # BN-backward prologue, ragged tail (M = 495)
    (3, 256, 13, 13, 128, 1, 3),    # prologue with the ReLU mask recomputed from Y2
    (64, 128, 14, 14, 128, 1, 0),   # one tile over 256 slices (M = 12544, slab sum of 196)
])
def test_conv1x1_wgrad_deep_shapes_match_fp32(b, cin, h, w, cout, s, pro):
    """The 128 x 128-tile weight gradient (layer 2-4 shape classes) against fp32 einsum, with the
    BN-backward prologue dY = k1·G + k2·Y2 + k3 (masked by Y2·s + t > 0 for pro = 3) formed while
    staging; ragged pixel tails and many slices; bitwise repeatable."""
    torch.manual_seed(6)
    x = _x(b, cin, h, w)
    oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
    like = torch.empty(cout, cin, 1, 1, device="cuda", dtype=torch.bfloat16)
    if pro:
        g, y2 = _x(b, cout, oh, ow), _x(b, cout, oh, ow)
        coef = torch.randn(5 if pro == 3 else 3, cout, device="cuda")
        v = lambda i: coef[i].view(1, -1, 1, 1)  # noqa: E731
        gm = torch.where(y2.float() * v(3) + v(4) > 0, g.float(), 0.0) if pro == 3 else g.float()
        dyf = (v(0) * gm + v(1) * y2.float() + v(2)).to(torch.bfloat16).float()
        dw = C.conv1x1_wgrad(g, x, 1, like, y2, coef)
    else:
        dy = _x(b, cout, oh, ow)
        dyf = dy.float()
        dw = C.conv1x1_wgrad(dy, x, s, like)
    ref = torch.einsum("bnhw,bkhw->nk", dyf, x.float()[:, :, ::s, ::s]).view(cout, cin, 1, 1)
    torch.testing.assert_close(dw.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    again = C.conv1x1_wgrad(g, x, 1, like, y2, coef) if pro else C.conv1x1_wgrad(dy, x, s, like)
    assert torch.equal(again, dw)  # fixed-order slab sum: bitwise deterministic


@pytest.mark.parametrize("offset", [0.0, 300.0])
def test_epilogue_stats_match_torch(offset):
    """Epilogue partials -> mean/var equal torch's over the stored bf16 output, also when
    |mean| >> std (shifted sums: no cancellation)."""
    torch.manual_seed(1)
    x = _x(4, 64, 20, 20, offset=offset)
    wt = (torch.randn(128, 64, 1, 1, device="cuda") / 8).to(torch.bfloat16)
    y, part = C.conv1x1_gemm(x, wt, 1, None, True)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 128)
    rm, rv = torch.zeros(128, device="cuda"), torch.ones(128, device="cuda")
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    mean, invstd, ss = C.bn_stats_from_partials(part, yf.shape[0], None, None, rm, rv, nbt, 0.1, False, 1e-5)
    var = yf.var(0, unbiased=False)
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-5, atol=1e-4 * yf.std(0).max().item())
    torch.testing.assert_close(1.0 / invstd ** 2 - 1e-5, var, rtol=2e-3, atol=1e-6)
    torch.testing.assert_close(rm, 0.1 * yf.mean(0), rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rv, 0.9 + 0.1 * yf.var(0, unbiased=True), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("b,cin,h,w,cout,masked", [(2, 64, 14, 14, 256, False), (3, 128, 9, 7, 64, False),
                                                   (2, 128, 10, 10, 128, True)])
def test_bn_backward_prologue_in_gemms(b, cin, h, w, cout, masked):
    """Input- and weight-gradient GEMMs forming dY = a·G + b·Y + c (G masked by Y·s + t > 0 when
    masked) while staging equal the plain GEMMs on the materialized dY."""
    torch.manual_seed(4)
    g, yb, x = _x(b, cout, h, w), _x(b, cout, h, w), _x(b, cin, h, w)
    coef = torch.randn(5 if masked else 3, cout, device="cuda")
    v = lambda i: coef[i].view(1, -1, 1, 1)  # noqa: E731
    gm = torch.where(yb.float() * v(3) + v(4) > 0, g.float(), 0.0) if masked else g.float()
    dy = (v(0) * gm + v(1) * yb.float() + v(2)).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(cin, cout, 1, 1, device="cuda") / cout ** 0.5).to(torch.bfloat16)  # [K_in, N_out] = W^T
    dx = C.conv1x1_gemm(g, wt, 1, coef, False, yb)[0]
    ref = C.conv1x1_gemm(dy, wt, 1, None, False)[0]
    torch.testing.assert_close(dx.float(), ref.float(), rtol=2e-2, atol=2e-2 * ref.float().abs().max().item())
    # the same GEMMs reading the forward weight W = [N_out, K_in] K-major (w_t): no transposed copy
    wf = wt.view(cin, cout).t().contiguous().view(cout, cin, 1, 1)
    dxt = C.conv1x1_gemm(g, wf, 1, coef, False, yb, True)[0]
    torch.testing.assert_close(dxt, dx, rtol=0, atol=0)
    reft = C.conv1x1_gemm(dy, wf, 1, None, False, None, True)[0]
    dref = F.conv_transpose2d(dy.float(), wf.float())  # dX = dY · W in fp32
    torch.testing.assert_close(reft.float(), dref, rtol=2e-2, atol=2e-2 * dref.abs().max().item())
    like = torch.empty(cout, cin, 1, 1, device="cuda", dtype=torch.float32)
    dw = C.conv1x1_wgrad(g, x, 1, like, yb, coef)
    refw = C.conv1x1_wgrad(dy, x, 1, like)
    torch.testing.assert_close(dw, refw, rtol=2e-2, atol=2e-2 * refw.abs().max().item())


@pytest.mark.parametrize("residual,relu,stride,cin", [(False, True, 1, 128), (True, True, 1, 128),
                                                      (False, False, 2, 128), (False, False, 1, 128),
                                                      (True, True, 1, 1024), (False, False, 1, 1024)])
def test_conv1x1_bn_act_forward_backward(residual, relu, stride, cin):
    """cin = 1024: the deep-K forward on the LDS-DMA GEMM with the statistics epilogue (group-minor
    partials, ops/conv_bn.py _DEEP_K)."""
    from distributeddataparallel_amd.ops import FusedBatchNorm2d, conv1x1_bn_act

    torch.manual_seed(2)
    conv = torch.nn.Conv2d(cin, 256, 1, stride=stride, bias=False).cuda().to(torch.bfloat16)
    bn = FusedBatchNorm2d(256).cuda().to(torch.bfloat16)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv = conv.to(memory_format=torch.channels_last)
    x = _x(4, cin, 12, 12).requires_grad_()
    oh = (12 - 1) // stride + 1
    res = _x(4, 256, oh, oh).requires_grad_() if residual else None
    out = conv1x1_bn_act(x, conv, bn, residual=res, relu=relu)
    g = torch.randn_like(out)
    out.backward(g)
    # fp32 reference of the same math
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().float().requires_grad_()
    gr, br = bn.weight.detach().float().requires_grad_(), bn.bias.detach().float().requires_grad_()
    rr = res.detach().float().requires_grad_() if residual else None
    yr = F.conv2d(xr, wr, stride=stride)
    yr = yr + (yr.to(torch.bfloat16).float() - yr).detach()  # the kernel normalizes the stored bf16 y
    o = F.batch_norm(yr, None, None, gr, br, True, 0.1, 1e-5)
    if residual:
        o = o + rr
    if relu:
        o = torch.relu(o)
    o.backward(g.float())
    tol = lambda ref: dict(rtol=3e-2, atol=3e-2 * ref.abs().max().item())  # noqa: E731
    torch.testing.assert_close(out.float(), o.detach(), **tol(o))

    # gradients: relative L2 error (a ReLU whose input rounds to ~0 may flip between bf16 and fp32
    # and move one pixel's gradient, so elementwise max error is not the right metric)
    def rel(a, b):
        return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()

    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(conv.weight.grad, wr.grad) < 2e-2
    assert rel(bn.weight.grad, gr.grad) < 2e-2
    assert rel(bn.bias.grad, br.grad) < 2e-2
    if residual:
        assert rel(res.grad, rr.grad) < 2e-2
    assert int(bn.num_batches_tracked) == 1


def test_bottleneck_resnet_conv_bn_fusion_matches_unfused(monkeypatch):
    """A bottleneck ResNet (one block per stage, every ResNet-50 block shape incl. the strided
    downsamples; bf16, channels_last): the fused 1x1-conv+BN path must be as close to an fp32 run of
    the same model as the unfused bf16 path is. (Each block alone agrees with the unfused path to
    ~1e-2, scripts/dbg/convbn_dbg2.py; through the stack both bf16 paths drift from fp32 alike.)"""
    from distributeddataparallel_amd.models.resnet import Bottleneck, ResNet
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    torch.manual_seed(3)
    m = ResNet(Bottleneck, [1, 1, 1, 1], norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last)
    x = torch.randn(8, 3, 96, 96, device="cuda").contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (8,), device="cuda")
    sd = {k: v.clone() for k, v in m.state_dict().items()}

    def run(dtype, flag):
        monkeypatch.setenv("XDDP_CONV_BN_FUSION", flag)
        m.load_state_dict(sd)
        mm = m.to(dtype)
        mm.zero_grad()
        loss = F.cross_entropy(mm(x.to(dtype)).float(), y)
        loss.backward()
        g = torch.cat([p.grad.float().flatten() for p in mm.parameters()])
        m.float()
        return loss.item(), g

    l32, g32 = run(torch.float32, "0")
    lf, gf = run(torch.bfloat16, "1")
    lu, gu = run(torch.bfloat16, "0")
    err = lambda g: ((g - g32).norm() / g32.norm()).item()  # noqa: E731
    assert abs(lf - l32) < 2e-2 * abs(l32) and abs(lu - l32) < 2e-2 * abs(l32)
    assert err(gf) < 1.5 * err(gu) + 0.02, (err(gf), err(gu))
    cos = lambda g: F.cosine_similarity(g, g32, dim=0).item()  # noqa: E731
    assert cos(gf) > cos(gu) - 0.02, (cos(gf), cos(gu))


@pytest.mark.parametrize("b,cin,h,w,cout", [(2, 64, 14, 14, 256), (3, 64, 9, 7, 128), (2, 128, 7, 7, 64),
                                             # K >= 256: the dense-GEMM pipeline (gemm.hip kEpiBnBwd)
                                             (2, 256, 14, 14, 1024), (3, 512, 7, 7, 256)])
def test_dgrad_bn_reduce_epilogue(b, cin, h, w, cout):
    """Input-gradient GEMM with the EPI epilogue: g = mask·(dY·W + add) stored, and per-channel
    (sum g, sum g·(y - mean)) partials, against fp32 PyTorch of the same math."""
    torch.manual_seed(5)
    dy = _x(b, cin, h, w)  # gradient at the conv1 output: [M, N_out = cin]
    wf = (torch.randn(cin, cout, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)  # W[N_out, K_in = cout]
    add, yb = _x(b, cout, h, w), _x(b, cout, h, w, offset=0.3)
    keep = torch.rand(b, cout, h, w, device="cuda") > 0.4
    flat = keep.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.int32)
    bits = (flat << torch.arange(8, device="cuda", dtype=torch.int32)).sum(1).to(torch.uint8)
    mean = yb.float().mean((0, 2, 3))
    g, part = C.conv1x1_gemm(dy, wf, 1, None, False, None, True, add, yb, bits, mean)
    ref = torch.where(keep, F.conv_transpose2d(dy.float(), wf.float()) + add.float(), 0.0)
    torch.testing.assert_close(g.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    assert part.dim() == 3 and part.size(1) == cout and part.size(2) == 2
    sd, sdx = part.sum(0).unbind(1)
    gq = g.float()
    torch.testing.assert_close(sd, gq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(sdx, (gq * (yb.float() - mean.view(1, -1, 1, 1))).sum((0, 2, 3)), rtol=1e-3,
                               atol=1e-2)
    # finalize: (k1, k2, k3 - k2·mean) and (dweight, dbias) of the previous BN
    weight = torch.rand(cout, device="cuda") + 0.5
    invstd = torch.rand(cout, device="cuda") + 0.5
    M = b * h * w
    coef, dwt, dbs = C.bn_backward_from_partials(part, M, weight, mean, invstd, True, True)
    torch.testing.assert_close(dbs, sd, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dwt, sdx * invstd, rtol=1e-4, atol=1e-4)
    k1, k2 = weight * invstd, -weight * invstd ** 3 * sdx / M
    k3 = -weight * invstd * sd / M - k2 * mean
    torch.testing.assert_close(coef, torch.stack([k1, k2, k3]), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("b,cin,h,w,cout", [(2, 64, 14, 14, 256), (2, 128, 7, 9, 128), (2, 256, 14, 14, 512),
                                             (2, 256, 7, 9, 256)])
def test_dgrad_bn_reduce_epilogue_stride2_add(b, cin, h, w, cout):
    """EPI epilogue with the compact stride-2 addend (a downsample's input gradient, only at the
    even (h, w) pixels), against fp32 PyTorch of the same math."""
    torch.manual_seed(7)
    dy = _x(b, cin, h, w)
    wf = (torch.randn(cin, cout, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
    add = _x(b, cout, (h + 1) // 2, (w + 1) // 2)
    yb = _x(b, cout, h, w, offset=0.3)
    keep = torch.rand(b, cout, h, w, device="cuda") > 0.4
    flat = keep.permute(0, 2, 3, 1).reshape(-1, 8).to(torch.int32)
    bits = (flat << torch.arange(8, device="cuda", dtype=torch.int32)).sum(1).to(torch.uint8)
    mean = yb.float().mean((0, 2, 3))
    g, part = C.conv1x1_gemm(dy, wf, 1, None, False, None, True, add, yb, bits, mean, None, 2)
    full = torch.zeros(b, cout, h, w, device="cuda")
    full[:, :, ::2, ::2] = add.float()
    ref = torch.where(keep, F.conv_transpose2d(dy.float(), wf.float()) + full, 0.0)
    torch.testing.assert_close(g.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    sd, sdx = part.sum(0).unbind(1)
    gq = g.float()
    torch.testing.assert_close(sd, gq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(sdx, (gq * (yb.float() - mean.view(1, -1, 1, 1))).sum((0, 2, 3)), rtol=1e-3,
                               atol=1e-2)


def test_downsample_epilogue_handoff_matches_separate_pass(monkeypatch):
    """Stride-2 downsample blocks fed by a linked block output: the downsample's compact input
    gradient folded into conv1's epilogue (XDDP_CONV_EPI_DS=1) gives the same gradients as the
    scattered full-resolution gradient + the producer's own reduce pass (=0)."""
    from distributeddataparallel_amd.models.resnet import Bottleneck, ResNet
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)  # (see the DeferredBN test)
    # (bitwise-identical forwards: the pending-apply GEMM's statistics tiles differ from the plain one's)
    monkeypatch.setenv("XDDP_PENDING_APPLY", "0")
    torch.manual_seed(8)
    m = ResNet(Bottleneck, [1, 1, 2, 1], norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16)
    m = m.to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 96, 96, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (4,), device="cuda")
    sd = {k: v.clone() for k, v in m.state_dict().items()}

    def run(flag):
        monkeypatch.setenv("XDDP_CONV_EPI_DS", flag)
        m.load_state_dict(sd)
        m.zero_grad()
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        return loss.item(), torch.cat([p.grad.float().flatten() for p in m.parameters()])

    l1, g1 = run("1")
    l0, g0 = run("0")
    assert abs(l1 - l0) < 1e-6 * max(1.0, abs(l0))
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-2
    assert F.cosine_similarity(g1, g0, dim=0).item() > 0.999


def test_downsample_bn_deferred_into_final_apply(monkeypatch):
    """The downsample's BN apply folded into the block's final apply pass (XDDP_DS_DEFER=1,
    ops/conv_bn.py:DeferredBN) gives the same loss, gradients, running statistics and
    num_batches_tracked as the downsample's own apply pass (=0)."""
    from distributeddataparallel_amd.models.resnet import Bottleneck, ResNet
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    # MIOpen's stride-2 3x3 gradients pick between algorithms from call to call, and at batch 4
    # the BN backward of the 3x3-pixel layer4 amplifies their rounding differences by 10-100x
    # (two runs of the SAME mode differed by up to 7 %): deterministic algorithms for the A/B
    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)
    torch.manual_seed(9)
    m = ResNet(Bottleneck, [1, 2, 1, 1], norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16)
    m = m.to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 96, 96, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (4,), device="cuda")
    sd = {k: v.clone() for k, v in m.state_dict().items()}

    def run(flag):
        monkeypatch.setenv("XDDP_DS_DEFER", flag)
        m.load_state_dict(sd)
        m.zero_grad()
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        bufs = {k: v.clone() for k, v in m.state_dict().items() if "running" in k or "num_batches" in k}
        return loss.item(), torch.cat([p.grad.float().flatten() for p in m.parameters()]), bufs

    l1, g1, b1 = run("1")
    l0, g0, b0 = run("0")
    assert abs(l1 - l0) < 2e-3 * max(1.0, abs(l0))
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-2
    assert F.cosine_similarity(g1, g0, dim=0).item() > 0.999
    for k in b0:
        torch.testing.assert_close(b1[k].float(), b0[k].float(), rtol=1e-2, atol=1e-3)
    assert int(b1["layer2.0.downsample.1.num_batches_tracked"]) == 1


def test_bottleneck_epilogue_handoff_matches_separate_pass(monkeypatch):
    """ResNet with two bottlenecks in a stage (so one block output feeds a non-downsample block):
    the conv1-epilogue hand-off of the previous block's BN backward (XDDP_CONV_EPI=1) gives the
    same gradients as the separate reduce pass (=0)."""
    from distributeddataparallel_amd.models.resnet import Bottleneck, ResNet
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    monkeypatch.setattr(torch.backends.cudnn, "deterministic", True)  # (see the DeferredBN test)
    # (bitwise-identical forwards: the pending-apply GEMM's statistics tiles differ from the plain one's)
    monkeypatch.setenv("XDDP_PENDING_APPLY", "0")
    torch.manual_seed(6)
    m = ResNet(Bottleneck, [2, 2, 1, 1], norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16)
    m = m.to(memory_format=torch.channels_last)
    x = torch.randn(4, 3, 64, 64, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (4,), device="cuda")
    sd = {k: v.clone() for k, v in m.state_dict().items()}

    def run(flag):
        monkeypatch.setenv("XDDP_CONV_EPI", flag)
        m.load_state_dict(sd)
        m.zero_grad()
        loss = F.cross_entropy(m(x).float(), y)
        loss.backward()
        return loss.item(), torch.cat([p.grad.float().flatten() for p in m.parameters()])

    l1, g1 = run("1")
    l0, g0 = run("0")
    assert abs(l1 - l0) < 1e-6 * max(1.0, abs(l0))
    assert ((g1 - g0).norm() / g0.norm()).item() < 2e-2
    assert F.cosine_similarity(g1, g0, dim=0).item() > 0.999


@pytest.mark.parametrize("pro", [False, True])
@pytest.mark.parametrize("b,cin,h,w,cout", [(2, 256, 14, 14, 64), (3, 128, 9, 7, 128), (2, 64, 8, 8, 256)])
def test_dgrad_bn_mask_recompute_epilogue(pro, b, cin, h, w, cout):
    """EPI second form (conv3 input gradient -> BN2 backward): g = [relu(y2·s + t) > 0]·dX with
    dX = dY·W (optionally dY = k1·g3 + k2·y3 + k3 formed in the prologue), stored, plus per-channel
    (sum g, sum g·(y2 - mean)) partials — against fp32 PyTorch of the same math."""
    torch.manual_seed(7)
    dy = _x(b, cin, h, w)
    wf = (torch.randn(cin, cout, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
    y2 = _x(b, cout, h, w, offset=0.2)
    ss = torch.stack([torch.rand(cout, device="cuda") + 0.5, torch.randn(cout, device="cuda") * 0.3]).contiguous()
    mean = y2.float().mean((0, 2, 3))
    if pro:
        y3 = _x(b, cin, h, w, offset=-0.1)
        coef = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda") * 0.1,
                            torch.randn(cin, device="cuda") * 0.05]).contiguous()
        g, part = C.conv1x1_gemm(dy, wf, 1, coef, False, y3, True, None, y2, None, mean, ss)
        src = (coef[0].view(1, -1, 1, 1) * dy.float() + coef[1].view(1, -1, 1, 1) * y3.float()
               + coef[2].view(1, -1, 1, 1)).to(torch.bfloat16).float()
    else:
        g, part = C.conv1x1_gemm(dy, wf, 1, None, False, None, True, None, y2, None, mean, ss)
        src = dy.float()
    keep = (y2.float() * ss[0].view(1, -1, 1, 1) + ss[1].view(1, -1, 1, 1)) > 0
    ref = torch.where(keep, F.conv_transpose2d(src, wf.float()), 0.0)
    torch.testing.assert_close(g.float(), ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item())
    sd, sdx = part.sum(0).unbind(1)
    gq = g.float()
    torch.testing.assert_close(sd, gq.sum((0, 2, 3)), rtol=1e-3, atol=1e-2)
    torch.testing.assert_close(sdx, (gq * (y2.float() - mean.view(1, -1, 1, 1))).sum((0, 2, 3)), rtol=1e-3,
                               atol=1e-2)
    # the unfolded finalize + elementwise pass = the full BN backward on the masked gradient
    weight = torch.rand(cout, device="cuda") + 0.5
    invstd = torch.rand(cout, device="cuda") + 0.5
    M = b * h * w
    coef2, _, _ = C.bn_backward_from_partials(part, M, weight, mean, invstd, False, False)
    dx = C.bn_backward_elem(g, y2, mean, coef2)
    xh = (y2.float() - mean.view(1, -1, 1, 1)) * invstd.view(1, -1, 1, 1)
    want = weight.view(1, -1, 1, 1) * invstd.view(1, -1, 1, 1) * (
        gq - (sd / M).view(1, -1, 1, 1) - xh * (sdx * invstd / M).view(1, -1, 1, 1))
    torch.testing.assert_close(dx.float(), want, rtol=2e-2, atol=2e-2 * want.abs().max().item())


@pytest.mark.parametrize("N,K,pro", [(256, 64, 2), (256, 64, 3), (64, 256, 2), (64, 256, 3)])
def test_conv1x1_bwd_fused_matches_separate_kernels(N, K, pro):
    """conv1x1_bwd_fused (dgrad + wgrad from one staging of dY = k1·g + k2·y2 + k3') equals the
    separate dgrad GEMM + wgrad kernel on the same prologue, and the fp32 math of dY."""
    from distributeddataparallel_amd._native import load

    C = load()
    g = torch.Generator(device="cuda").manual_seed(5)
    B, H, W = 3, 55, 57  # M = 9405: a partial last 64-row step
    cl = torch.channels_last
    gr = torch.randn(B, N, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    y2 = torch.randn(B, N, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    x = torch.randn(B, K, H, W, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(N, K, 1, 1, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    rows = 5 if pro == 3 else 3
    coef = torch.randn(rows, N, device="cuda", generator=g) * 0.5
    if pro == 3:
        coef[3].abs_().add_(0.1)  # a positive BN scale for the mask recompute
    coef = coef.contiguous()
    dx_f, dw_f = C.conv1x1_bwd_fused(gr, y2, coef, x, w)
    dx_s = C.conv1x1_gemm(gr, w, 1, coef, False, y2, True)[0]
    dw_s = C.conv1x1_wgrad(gr, x, 1, w, y2, coef)

    def rel(a, b):
        return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()

    assert rel(dx_f, dx_s) < 5e-3, rel(dx_f, dx_s)
    assert rel(dw_f.view(N, K), dw_s.view(N, K)) < 5e-3, rel(dw_f.view(N, K), dw_s.view(N, K))
    # fp32 reference of the same math
    gf, yf = gr.float(), y2.float()
    if pro == 3:
        gf = torch.where(yf * coef[3].view(1, -1, 1, 1) + coef[4].view(1, -1, 1, 1) > 0, gf, torch.zeros_like(gf))
    dy = (coef[0].view(1, -1, 1, 1) * gf + coef[1].view(1, -1, 1, 1) * yf + coef[2].view(1, -1, 1, 1)).to(
        torch.bfloat16).float()
    dx_r = torch.einsum("bnhw,nk->bkhw", dy, w.float().view(N, K))
    dw_r = torch.einsum("bnhw,bkhw->nk", dy, x.float())
    assert rel(dx_f, dx_r) < 1e-2 and rel(dw_f.view(N, K), dw_r) < 1e-2
