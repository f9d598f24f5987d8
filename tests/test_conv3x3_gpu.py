"""3x3 implicit-GEMM conv (csrc/kernels/conv3x3.hip): forward, BN-statistics epilogue, rotated
weights for the stride-1 input gradient, and the fused conv3x3+BN+ReLU op — against plain
PyTorch fp32 references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

from distributeddataparallel_amd._native import load

pytestmark = pytest.mark.gpu

C = load() if torch.cuda.is_available() else None


def _cl(t):
    return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


@pytest.mark.parametrize("b,cin,h,w,cout,s,off", [
    (2, 64, 14, 14, 64, 1, 0.0),     # N = 64 tile, M = 392: partial last M-tile
    (3, 128, 9, 7, 128, 1, 30.0),    # odd spatial size, 256x128 tile, |mean| >> std per channel
    (2, 64, 15, 15, 256, 2, 0.0),    # strided, odd input size
    (1, 512, 7, 7, 512, 1, 0.0),     # long reduction (72 steps), one M-tile
    (8, 64, 40, 40, 64, 1, 0.0),     # 100 M-tiles: many stats partials
    # N >= 256: the dense-GEMM pipeline with im2col addressing (gemm.hip ConvGeo)
    (3, 256, 14, 14, 256, 1, 30.0),  # layer-3 shape, partial last 256-row tile, |mean| >> std
    (2, 128, 9, 11, 384, 1, 0.0),    # three 128-wide N tiles, odd spatial size
    (2, 256, 15, 13, 256, 2, 0.0),   # strided, odd input size
    (2, 192, 8, 8, 256, 1, 0.0),     # C / 64 = 3 (not a power of two): the conv3x3.hip kernel
    # stride 1, W = 56 / 28 / 14: the row-band kernel (conv3x3_band.hip)
    (2, 64, 56, 56, 64, 1, 30.0),    # layer-1 shape: 4-row bands
    (2, 128, 28, 28, 128, 1, 0.0),   # layer-2 shape: two 64-channel steps, 7-row bands
    (3, 128, 17, 23, 64, 1, 0.0),    # odd width: the conv3x3.hip kernel
    (1, 64, 15, 130, 64, 1, 0.0),    # W > 128: the conv3x3.hip kernel
])
def test_conv3x3_forward_matches_conv2d(b, cin, h, w, cout, s, off):
    torch.manual_seed(0)
    x = _cl(torch.randn(b, cin, h, w, device="cuda") + off)
    wt = _cl(torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5)
    y, part = C.conv3x3_forward(x, wt, s, True)
    ref = F.conv2d(x.float(), wt.float(), stride=s, padding=1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    # epilogue statistics of the stored bf16 output
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, cout)
    rm, rv = torch.zeros(cout, device="cuda"), torch.ones(cout, device="cuda")
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    mean, invstd, _ = C.bn_stats_from_partials(part, yf.shape[0], None, None, rm, rv, nbt, 0.1, False, 1e-5, True)
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-5, atol=1e-4 * yf.std(0).max().item())
    torch.testing.assert_close(1.0 / invstd ** 2 - 1e-5, yf.var(0, unbiased=False), rtol=2e-3, atol=1e-6)


@pytest.mark.parametrize("cin,cout,h,w", [(128, 64, 10, 11), (256, 256, 10, 11), (64, 64, 20, 30), (128, 128, 14, 14)])
def test_conv3x3_rotated_weight_gives_input_gradient(cin, cout, h, w):
    torch.manual_seed(1)
    x = torch.randn(2, cin, h, w, device="cuda")
    wt = torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5
    dy = torch.randn(2, cout, h, w, device="cuda")
    rot = C.conv3x3_rot_weight(_cl(wt))
    torch.testing.assert_close(rot.float(), _cl(wt).float().flip(2, 3).transpose(0, 1), rtol=0, atol=0)
    dx = C.conv3x3_forward(_cl(dy), rot, 1, False)[0]
    xr = x.to(torch.bfloat16).float().requires_grad_()
    F.conv2d(xr, _cl(wt).float(), padding=1).backward(_cl(dy).float())
    torch.testing.assert_close(dx.float(), xr.grad, rtol=1e-2, atol=1e-2 * xr.grad.abs().max().item())


def test_conv3x3_rot_weights_batched_matches_single():
    """One launch over several weights (40 > one 32-tensor batch) equals the per-tensor rotation."""
    torch.manual_seed(4)
    ws = [_cl(torch.randn(64 * (1 + i % 4), 64 * (1 + (i // 4) % 3), 3, 3, device="cuda")) for i in range(40)]
    outs = C.conv3x3_rot_weights(ws)
    for w, o in zip(ws, outs):
        assert torch.equal(o, C.conv3x3_rot_weight(w))


def test_conv3x3_rotated_weights_follow_in_place_updates():
    """The backward's rotated weights are recomputed after every forward (the fused optimizers
    write parameter memory in place without bumping the tensor version): two steps with an
    in-place weight change in between give the same input gradients as fresh modules."""
    from distributeddataparallel_amd.ops import FusedBatchNorm2d, conv3x3_bn_relu

    torch.manual_seed(5)
    conv = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).cuda().to(torch.bfloat16).to(
        memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(64).cuda().to(torch.bfloat16)
    bn.relu = True
    x = _cl(torch.randn(2, 64, 12, 12, device="cuda")).requires_grad_()
    g = torch.randn(2, 64, 12, 12, device="cuda", dtype=torch.bfloat16)
    for step in range(2):
        x.grad = None
        conv3x3_bn_relu(x, conv, bn).backward(g)
        got = x.grad.clone()
        ref_conv = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).cuda().to(torch.bfloat16).to(
            memory_format=torch.channels_last)
        ref_bn = FusedBatchNorm2d(64).cuda().to(torch.bfloat16)
        ref_bn.relu = True
        ref_conv.load_state_dict(conv.state_dict())
        ref_bn.load_state_dict(bn.state_dict())
        xr = x.detach().clone().requires_grad_()
        ref_bn.train()
        with torch.no_grad():  # the same batch statistics: start from bn's pre-step running stats
            ref_bn.running_mean.copy_(bn.running_mean)
        conv3x3_bn_relu(xr, ref_conv, ref_bn).backward(g)
        assert torch.equal(got, xr.grad), step
        with torch.no_grad():
            conv.weight.data.mul_(-0.5).add_(0.01)  # an in-place update the next step must see


@pytest.mark.parametrize("b,cin,h,w,cout", [
    (2, 128, 10, 11, 64),    # odd width: phase grids of unequal size
    (3, 64, 15, 15, 128),    # odd input: the last dY row/column feeds the even phase only
    (2, 128, 28, 28, 128),   # ResNet-50 layer2 entry shape (reduced batch), 256x128 tiles
    (1, 512, 14, 14, 512),   # layer4 entry shape, long reduction
    (2, 256, 28, 28, 256),   # layer3 entry shape
    (1, 128, 56, 56, 128),   # layer2 entry spatial size
    (1, 128, 6, 10, 64),     # 15 dY pixels: one partial m-tile per phase, Cout 64 (1-K-tile phase)
])
def test_conv3x3_dgrad_s2_matches_conv2d(b, cin, h, w, cout):
    """Stride-2 input gradient over the four phase grids vs fp32 autograd: even input sizes with
    Cin % 128 == 0 run the four phase GEMMs on the dense GEMM pipeline (gemm.hip DGS2), the odd
    ones the phase-grid kernel (conv3x3.hip DG2)."""
    torch.manual_seed(3)
    x = torch.randn(b, cin, h, w, device="cuda")
    wt = torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    dy = _cl(torch.randn(b, cout, oh, ow, device="cuda"))
    dx = C.conv3x3_dgrad_s2(dy, C.conv3x3_rot_weight(_cl(wt)), h, w)
    xr = x.requires_grad_()
    F.conv2d(xr, _cl(wt).float(), stride=2, padding=1).backward(dy.float())
    assert dx.shape == xr.shape and dx.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(dx.float(), xr.grad, rtol=1e-2, atol=1e-2 * xr.grad.abs().max().item())


@pytest.mark.parametrize("stride", [1, 2])
def test_conv3x3_bn_relu_forward_backward(stride):
    from distributeddataparallel_amd.ops import FusedBatchNorm2d, conv3x3_bn_relu

    torch.manual_seed(2)
    conv = torch.nn.Conv2d(64, 128, 3, stride=stride, padding=1, bias=False).cuda().to(torch.bfloat16)
    conv = conv.to(memory_format=torch.channels_last)
    bn = FusedBatchNorm2d(128).cuda().to(torch.bfloat16)
    bn.relu = True
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    x = _cl(torch.randn(4, 64, 13, 13, device="cuda")).requires_grad_()
    out = conv3x3_bn_relu(x, conv, bn)
    g = torch.randn_like(out)
    out.backward(g)
    xr = x.detach().float().requires_grad_()
    wr = conv.weight.detach().float().requires_grad_()
    gr, br = bn.weight.detach().float().requires_grad_(), bn.bias.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, stride=stride, padding=1)
    yr = yr + (yr.to(torch.bfloat16).float() - yr).detach()  # the kernel normalizes the stored bf16 y
    o = torch.relu(F.batch_norm(yr, None, None, gr, br, True, 0.1, 1e-5))
    o.backward(g.float())
    torch.testing.assert_close(out.float(), o.detach(), rtol=3e-2, atol=3e-2 * o.abs().max().item())

    def rel(a, b):
        return ((a.float() - b).norm() / (b.norm() + 1e-12)).item()

    assert rel(x.grad, xr.grad) < 2e-2
    assert rel(conv.weight.grad, wr.grad) < 2e-2
    assert rel(bn.weight.grad, gr.grad) < 2e-2
    assert rel(bn.bias.grad, br.grad) < 2e-2
    assert int(bn.num_batches_tracked) == 1


@pytest.mark.parametrize("b,cin,h,w,cout,s", [
    (2, 64, 16, 16, 64, 1),     # exact 8x8 patch grid
    (3, 64, 14, 14, 128, 1),    # partial patches (14 = 8 + 6), 2 n-tiles
    (2, 128, 9, 7, 64, 1),      # odd spatial size, 2 c-tiles
    (2, 64, 15, 15, 64, 2),     # strided, odd input size (phase-split halo)
    (2, 128, 28, 28, 128, 2),   # strided, ResNet-50 layer2 entry shape (reduced batch): 128-channel n tiles
    (2, 256, 14, 14, 256, 2),   # strided, layer3 entry shape: 2 x 4 tiles of 128 x 64
    (1, 64, 16, 16, 128, 2),    # strided, N = 128 over a 64-channel input
    (1, 512, 7, 7, 512, 1),     # one partial patch per image, 64 tiles
    (4, 64, 56, 56, 64, 1),     # ResNet-50 layer1 shape (reduced batch): many splits
    (2, 64, 12, 20, 64, 1),     # non-square, partial last patch column
    (2, 128, 28, 28, 128, 1),   # layer2 shape (reduced batch)
])
def test_conv3x3_wgrad_patch_matches_conv2d(b, cin, h, w, cout, s):
    """8x8-patch 3x3 weight gradient (csrc/kernels/conv3x3_wgrad.hip) vs fp32 PyTorch."""
    torch.manual_seed(1)
    x = _cl(torch.randn(b, cin, h, w, device="cuda"))
    oh, ow = (h - 1) // s + 1, (w - 1) // s + 1
    dy = _cl(torch.randn(b, cout, oh, ow, device="cuda"))
    wt = _cl(torch.randn(cout, cin, 3, 3, device="cuda"))
    dw = C.conv3x3_wgrad_patch(dy, x, s, wt)
    assert dw.shape == wt.shape and dw.dtype == wt.dtype and dw.is_contiguous(memory_format=torch.channels_last)
    ref = torch.nn.grad.conv2d_weight(x.float(), wt.shape, dy.float(), stride=s, padding=1)
    torch.testing.assert_close(dw.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    # fp32 output: no bf16 rounding of the result, only the inputs' (exact products, fp32 sums)
    dw32 = C.conv3x3_wgrad_patch(dy, x, s, wt.float())
    torch.testing.assert_close(dw32, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())


@pytest.mark.parametrize("b,cin,h,w,cout", [
    (2, 64, 56, 56, 64),     # W = 56: 4-row bands inside one image
    (3, 128, 28, 28, 128),   # W = 28: 8-row bands, every 4th crosses two images; 84 rows -> a partial last band
    (5, 256, 14, 14, 128),   # W = 14: 16-row bands over 2-3 images, 2 n-tiles x 4 c-tiles
    (9, 128, 7, 7, 256),     # W = 7: 32-row bands over up to 6 images (halo segments), 63 rows -> partial
    (1, 64, 9, 7, 64),       # a single partial band (9 rows < R = 32)
])
def test_conv3x3_wgrad_band_matches_conv2d_and_patch(b, cin, h, w, cout):
    """Stride-1 weight gradient on 224-pixel row bands (conv3x3_wgrad_band_kernel, splits_req = -2; opt-in
    by XDDP_WGRAD3_BAND=1, slower than the patch kernel) vs fp32 PyTorch, and vs the 8x8-patch kernel
    (splits = 0) with fp32 output."""
    torch.manual_seed(7)
    x = _cl(torch.randn(b, cin, h, w, device="cuda"))
    dy = _cl(torch.randn(b, cout, h, w, device="cuda"))
    wt = _cl(torch.randn(cout, cin, 3, 3, device="cuda"))
    ref = torch.nn.grad.conv2d_weight(x.float(), wt.shape, dy.float(), stride=1, padding=1)
    band = C.conv3x3_wgrad_patch(dy, x, 1, wt.float(), -2)
    patch = C.conv3x3_wgrad_patch(dy, x, 1, wt.float(), 0)
    torch.testing.assert_close(band, ref, rtol=1e-4, atol=1e-4 * ref.abs().max().item())
    torch.testing.assert_close(band, patch, rtol=1e-5, atol=1e-5 * ref.abs().max().item())
    bb = C.conv3x3_wgrad_patch(dy, x, 1, wt, -2)
    assert bb.dtype == torch.bfloat16 and bb.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(bb.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    assert torch.equal(C.conv3x3_wgrad_patch(dy, x, 1, wt, -2), bb)  # fixed-order slab sum: bitwise repeatable


@pytest.mark.parametrize("b,cin,h,w,cout,rows,cfg,off", [
    (2, 64, 56, 56, 64, 4, 0, 30.0),     # layer-1 band: 4 rows = 224 pixels, N = 64 tiles, weight ring
    (3, 128, 28, 28, 128, 7, 1, 0.0),    # layer-2 band: 7 rows = 196 pixels, 208-row tile, B in registers
    (3, 128, 28, 28, 256, 7, 1, 0.0),    # two N tiles
    (2, 256, 7, 7, 256, 28, 1, 5.0),     # bands over four images, 4 channel steps
    (3, 256, 14, 14, 256, 14, 1, 0.0),   # layer-3: one band = one image, two N tiles
    (5, 512, 7, 7, 512, 28, 1, 0.0),     # a band spans four images; partial last band
    (3, 128, 7, 7, 256, 29, 1, 10.0),    # bands start mid-image: first segment partial, 5 segments
    (2, 64, 10, 12, 64, 3, 0, 0.0),      # ragged: 20 rows in bands of 3, crossing an image edge
    (40, 64, 56, 56, 64, 4, 0, 30.0),    # 560 bands on the persistent statistics blocks (two per CU):
                                         # uneven, some blocks sum two bands under one shift
    (1, 128, 5, 9, 128, 23, 1, 0.0),     # more rows per band than the batch has (one partial band)
])
def test_conv3x3_band_matches_conv2d(b, cin, h, w, cout, rows, cfg, off):
    """Row-band kernel (conv3x3_band.hip) with explicit band heights and configurations: bands
    crossing image edges, partial first segments and a partial last band, output and BN statistics
    partials."""
    torch.manual_seed(2)
    x = _cl(torch.randn(b, cin, h, w, device="cuda") + off)
    wt = _cl(torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5)
    y, part = C.conv3x3_band_forward(x, wt, True, rows, cfg)
    ref = F.conv2d(x.float(), wt.float(), padding=1)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=1e-2 * ref.abs().max().item())
    # one statistics group per band, or per persistent block (N = 64 with statistics: <= 2 per CU)
    assert part.shape[:2] == (3, cout) and 1 <= part.shape[2] <= (b * h + rows - 1) // rows
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, cout)
    rm, rv = torch.zeros(cout, device="cuda"), torch.ones(cout, device="cuda")
    nbt = torch.zeros((), dtype=torch.long, device="cuda")
    mean, invstd, _ = C.bn_stats_from_partials(part, yf.shape[0], None, None, rm, rv, nbt, 0.1, False, 1e-5, True)
    torch.testing.assert_close(mean, yf.mean(0), rtol=1e-5, atol=1e-4 * yf.std(0).max().item())
    torch.testing.assert_close(1.0 / invstd ** 2 - 1e-5, yf.var(0, unbiased=False), rtol=2e-3, atol=1e-6)
    y2, _ = C.conv3x3_band_forward(x, wt, False, rows, cfg)  # the no-statistics instance: same output
    assert torch.equal(y, y2)
