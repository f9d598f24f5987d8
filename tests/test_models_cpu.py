"""Model zoo (structure/param counts) and DDP over transformer models on the CPU backend."""
import pytest
import torch
import torch.nn.functional as F

from _dist_utils import run_ranks


def test_param_counts_match_reference_architectures():
    from distributeddataparallel_amd.models import llama3_8b, resnet18, resnet50, vit_l_16

    assert sum(p.numel() for p in resnet18().parameters()) == 11_689_512
    assert sum(p.numel() for p in resnet50().parameters()) == 25_557_032
    assert sum(p.numel() for p in vit_l_16().parameters()) == 304_326_632
    with torch.device("meta"):
        assert sum(p.numel() for p in llama3_8b().parameters()) == 8_030_261_248


def test_simplecnn_state_dict_keys_match_reference_layout():
    from distributeddataparallel_amd.models import SimpleCNN

    keys = list(SimpleCNN().state_dict().keys())
    assert keys[0] == "model.conv1.weight" and "model.fc.weight" in keys and len(keys) == 122


def test_fused_norm_modules_fall_back_on_cpu():
    from distributeddataparallel_amd.ops import FusedBatchNorm2d, FusedLayerNorm, FusedRMSNorm

    x = torch.randn(2, 8, 4, 4)
    bn, ref = FusedBatchNorm2d(8), torch.nn.BatchNorm2d(8)
    torch.testing.assert_close(bn(x, relu=True), F.relu(ref(x)))
    assert list(bn.state_dict()) == list(ref.state_dict())
    y = torch.randn(3, 16)
    torch.testing.assert_close(FusedLayerNorm(16)(y), F.layer_norm(y, (16,)))
    r = FusedRMSNorm(16)(y)
    torch.testing.assert_close(r, y * torch.rsqrt(y.pow(2).mean(-1, keepdim=True) + 1e-6))


def _w_transformer(rank, world, which):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.models import llama_tiny, vit_tiny

    torch.manual_seed(0)
    make = (lambda: llama_tiny()) if which == "llama" else (lambda: vit_tiny(num_classes=10))
    m = make()
    torch.manual_seed(0)
    base = make()
    ddp = xddp.DDP(m, bucket_cap_mb=0.05, first_bucket_cap_mb=0.01)
    g = torch.Generator().manual_seed(7)
    for _ in range(3):
        if which == "llama":
            x = torch.randint(0, 512, (2 * world, 16), generator=g)
            y = torch.randint(0, 512, (2 * world, 16), generator=g)
            lf = lambda o, t: F.cross_entropy(o.reshape(-1, o.shape[-1]), t.reshape(-1))  # noqa: E731
        else:
            x = torch.randn(2 * world, 3, 32, 32, generator=g)
            y = torch.randint(0, 10, (2 * world,), generator=g)
            lf = F.cross_entropy
        xs, ys = x[rank * 2:(rank + 1) * 2], y[rank * 2:(rank + 1) * 2]
        m.zero_grad()
        base.zero_grad()
        lf(ddp(xs), ys).backward()
        lf(base(x), y).backward()
        for (n, a), b in zip(m.named_parameters(), base.parameters()):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-4, atol=1e-5, msg=n)
    assert len(ddp.reducer.bucket_sizes_bytes()) > 1


@pytest.mark.parametrize("which", ["llama", "vit"])
def test_ddp_transformers(which):
    run_ranks(_w_transformer, world=2, args=(which,))


def test_global_avg_pool_matches_adaptive_avg_pool():
    """ops.pool.global_avg_pool: same values and gradient as flatten(AdaptiveAvgPool2d(1)), with a
    channels_last gradient (no NCHW -> NHWC transpose copy in backward)."""
    from distributeddataparallel_amd.ops.pool import global_avg_pool

    torch.manual_seed(0)
    x = torch.randn(3, 16, 7, 5).contiguous(memory_format=torch.channels_last).requires_grad_()
    x2 = x.detach().clone().requires_grad_()
    y, y2 = global_avg_pool(x), torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x2, 1), 1)
    g = torch.randn_like(y)
    y.backward(g)
    y2.backward(g)
    torch.testing.assert_close(y, y2)
    torch.testing.assert_close(x.grad, x2.grad)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
