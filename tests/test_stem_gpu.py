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
