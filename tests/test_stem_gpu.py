"""Fused ResNet stem bn1 -> ReLU -> maxpool(3, 2, 1) (ops/pool.py: stem_bn_relu_maxpool, kernels
stem_pool_fwd / stem_pool_bn_bwd in csrc/kernels/pool.hip) vs an fp32 torch reference of the same
op, forward (pooled values, running stats) and backward (dx, dgamma, dbeta), with the dual output
(two consumers) of the ResNet stem; odd spatial sizes exercise the partial 2x2 quads. dx is held
tightly to the unfused bf16 kernels (same rounding, same first-max tie rule) and loosely to fp32:
pooling bf16-rounded values creates argmax ties that fp32 breaks differently, which routes a
window's whole gradient to another pixel (~5 % relative L2 at these shapes)."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(4, 64, 56, 56), (3, 64, 29, 31)])
def test_stem_bn_relu_maxpool_matches_fp32(shape):
    from distributeddataparallel_amd.ops import FusedBatchNorm2d
    from distributeddataparallel_amd.ops.pool import FusedMaxPool2d, _StemBNPool, stem_bn_relu_maxpool

    g = torch.Generator(device="cuda").manual_seed(3)
    N, C, H, W = shape
    y = (torch.randn(N, C, H, W, device="cuda", generator=g) * 2 + 0.3).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    d1 = torch.randn(N, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1, device="cuda", generator=g).to(torch.bfloat16)
    d2 = torch.randn(d1.shape, device="cuda", generator=g).to(torch.bfloat16)
    weight = (torch.rand(C, device="cuda", generator=g) - 0.3)  # some negative gammas: BN is not monotonic
    bias = torch.randn(C, device="cuda", generator=g) * 0.5

    bn = FusedBatchNorm2d(C).cuda()
    bn.relu = True
    with torch.no_grad():
        bn.weight.copy_(weight)
        bn.bias.copy_(bias)
    pool = FusedMaxPool2d(3, 2, 1)
    yin = y.clone().requires_grad_(True)
    calls = []
    orig = _StemBNPool.forward
    _StemBNPool.forward = staticmethod(lambda *a, **k: calls.append(1) or orig(*a, **k))
    try:
        out, out2 = stem_bn_relu_maxpool(yin, bn, pool, dual=True)
    finally:
        _StemBNPool.forward = staticmethod(orig)
    assert calls
    torch.autograd.backward([out, out2], [d1.contiguous(memory_format=torch.channels_last),
                                          d2.contiguous(memory_format=torch.channels_last)])

    ref = nn.BatchNorm2d(C).cuda()
    with torch.no_grad():
        ref.weight.copy_(weight)
        ref.bias.copy_(bias)
    yr = y.float().requires_grad_(True)
    o = F.max_pool2d(F.relu(ref(yr)), 3, 2, 1)
    o.backward(d1.float() + d2.float())

    def rel(a, b):
        return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()

    # the unfused xddp bf16 path: FusedBatchNorm2d(relu) -> FusedMaxPool2d (dual output)
    bn_u = FusedBatchNorm2d(C).cuda()
    bn_u.relu = True
    with torch.no_grad():
        bn_u.weight.copy_(weight)
        bn_u.bias.copy_(bias)
    pool_u = FusedMaxPool2d(3, 2, 1)
    pool_u.dual_output = True
    yu = y.clone().requires_grad_(True)
    ou, ou2 = pool_u(bn_u(yu))
    torch.autograd.backward([ou, ou2], [d1.contiguous(memory_format=torch.channels_last),
                                        d2.contiguous(memory_format=torch.channels_last)])

    assert rel(out, o) < 1e-2
    assert rel(out, ou) < 1e-3
    assert rel(yin.grad, yu.grad) < 1e-2, rel(yin.grad, yu.grad)
    assert rel(yin.grad, yr.grad) < 0.1, rel(yin.grad, yr.grad)
    assert rel(bn.weight.grad, bn_u.weight.grad) < 1e-2
    assert rel(bn.weight.grad, ref.weight.grad) < 2e-2
    assert rel(bn.bias.grad, ref.bias.grad) < 2e-2
    assert rel(bn.running_mean, ref.running_mean) < 1e-4
    assert rel(bn.running_var, ref.running_var) < 1e-3
    assert int(bn.num_batches_tracked) == 1


@pytest.mark.parametrize("shape", [(4, 3, 224, 224), (2, 3, 57, 61)])
def test_stem_conv_forward_and_wgrad_match_fp32(shape):
    """stem_conv_forward (output + BN-statistics partials) and stem_conv_wgrad vs fp32 torch."""
    from distributeddataparallel_amd._native import load

    C = load()
    g = torch.Generator(device="cuda").manual_seed(11)
    x = torch.randn(shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(64, 3, 7, 7, device="cuda", generator=g) * 0.1).to(torch.bfloat16)
    w_cl = w.contiguous(memory_format=torch.channels_last)  # the model's weights are channels_last
    y, part = C.stem_conv_forward(x, w_cl)
    yr = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    assert y.shape == yr.shape and y.is_contiguous(memory_format=torch.channels_last)

    def rel(a, b):
        return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()

    assert rel(y, yr) < 5e-3, rel(y, yr)
    M = y.numel() // 64
    mean, invstd, _ = C.bn_stats_from_partials(part, M, None, None, None, None, None, 0.0, False, 1e-5)
    var_r, mean_r = torch.var_mean(y.float(), dim=(0, 2, 3), unbiased=False)
    assert (mean - mean_r).abs().max().item() < 1e-3 * (var_r.sqrt().max().item() + 1)
    assert rel(1.0 / invstd ** 2 - 1e-5, var_r) < 1e-3

    dy = torch.randn(y.shape, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dw = C.stem_conv_wgrad(dy, x, w_cl)
    dwr = torch.nn.grad.conv2d_weight(x.float(), w.shape, dy.float(), stride=2, padding=3)
    assert dw.shape == w.shape and dw.dtype == w.dtype
    assert rel(dw, dwr) < 1e-2, rel(dw, dwr)


def test_resnet_stem_matches_unfused_stack():
    """The whole own-kernel stem (ops/stem.py) vs the same model stem on MIOpen conv + the
    unfused xddp BN / max-pool kernels: outputs and every parameter gradient."""
    import os

    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d
    from distributeddataparallel_amd.ops.stem import _Stem

    torch.manual_seed(0)
    m = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(8, 3, 112, 112, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)

    def stem_run(env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            for p in (m.conv1.weight, m.bn1.weight, m.bn1.bias):
                p.grad = None
            calls = []
            orig = _Stem.forward
            _Stem.forward = staticmethod(lambda *a, **k: calls.append(1) or orig(*a, **k))
            try:
                out = m.maxpool(m.relu(m.bn1(m.conv1(x)))) if env.get("XDDP_STEM_FUSION") == "0" else None
                if out is None:
                    fused = type(m).forward  # run only the stem part of ResNet.forward
                    del fused
                    from distributeddataparallel_amd.ops.stem import resnet_stem, stem_supported

                    if env.get("XDDP_STEM_CONV", "1") == "1":
                        assert stem_supported(x, m.conv1, m.bn1, m.maxpool)
                        out = resnet_stem(x, m.conv1, m.bn1, m.maxpool, dual=True)
                    else:
                        from distributeddataparallel_amd.ops.pool import stem_bn_relu_maxpool

                        out = stem_bn_relu_maxpool(m.conv1(x), m.bn1, m.maxpool, dual=True)
            finally:
                _Stem.forward = staticmethod(orig)
            o = out if isinstance(out, tuple) else (out,)
            torch.autograd.backward(list(o), [torch.ones_like(t) * 0.01 for t in o])
            return (o[0].float().clone(), m.conv1.weight.grad.float().clone(), m.bn1.weight.grad.float().clone(),
                    m.bn1.bias.grad.float().clone(), len(calls))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    own = stem_run({"XDDP_STEM_CONV": "1"})
    ref = stem_run({"XDDP_STEM_CONV": "0"})
    assert own[4] == 1 and ref[4] == 0

    def rel(a, b):
        return ((a - b).norm() / (b.norm() + 1e-12)).item()

    assert rel(own[0], ref[0]) < 2e-2
    for a, b in zip(own[1:4], ref[1:4]):
        assert rel(a, b) < 5e-2, rel(a, b)
