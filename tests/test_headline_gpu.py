"""Headline-config correctness (VERDICT r1 "Next round" #3): the bf16 channels_last ResNet-50 with
FusedBatchNorm2d — every fused path on (1x1-conv MFMA GEMM with BN-stats epilogue, 3x3 implicit
GEMM, EpiLink hand-off, BN-backward folded into the gradient GEMM prologues, own max-pool) — at a
real shape (224x224) against an fp32 torch model (nn.BatchNorm2d + MIOpen convs) from identical
weights.

Tolerances are self-calibrating: the same bf16 model run through plain torch ops (nn.BatchNorm2d,
MIOpen bf16 convs) is the yardstick of what bf16 rounding alone costs. The fused stack must stay
within a small factor of that yardstick, per parameter and overall.
"""
import os

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _counting(C, names):
    """Wrap native entry points with call counters (proves which kernels the model ran)."""
    counts = {n: 0 for n in names}
    orig = {n: getattr(C, n) for n in names}

    def wrap(n):
        def f(*a, **k):
            counts[n] += 1
            if n == "conv1x1_gemm" and len(a) > 7 and a[7] is not None:
                counts["epilink"] = counts.get("epilink", 0) + 1
            return orig[n](*a, **k)
        return f

    for n in names:
        setattr(C, n, wrap(n))
    return counts, orig


def _grad_stats(model, ref):
    out = {}
    for (n, p), q in zip(model.named_parameters(), ref.parameters()):
        a, b = p.grad.float().flatten(), q.grad.float().flatten()
        rel = ((a - b).norm() / (b.norm() + 1e-20)).item()
        cos = F.cosine_similarity(a, b, dim=0).item()
        out[n] = (rel, cos)
    return out


def _models(batch, size, seed=0, branch_gamma=None):
    from distributeddataparallel_amd.models import resnet50
    from distributeddataparallel_amd.ops import FusedBatchNorm2d

    torch.manual_seed(seed)
    fused = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    if branch_gamma is not None:  # SkipInit-style down-weighted residual branches (see below)
        with torch.no_grad():
            for name, mod in fused.named_modules():
                if name.endswith("bn3"):
                    mod.weight.fill_(branch_gamma)
    sd = {k: (v.float() if v.is_floating_point() else v) for k, v in fused.state_dict().items()}
    ref32 = resnet50().cuda().to(memory_format=torch.channels_last)
    ref32.load_state_dict(sd)
    ref16 = resnet50().cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref16.load_state_dict(fused.state_dict())
    g = torch.Generator(device="cuda").manual_seed(seed + 1)
    x16 = torch.randn(batch, 3, size, size, device="cuda", generator=g).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (batch,), device="cuda", generator=g)
    return fused, ref32, ref16, x16, y


def _run_three(batch, size, branch_gamma=None):
    from distributeddataparallel_amd._native import load

    C = load()
    fused, ref32, ref16, x16, y = _models(batch, size, branch_gamma=branch_gamma)
    counts, orig = _counting(C, ["conv1x1_gemm", "conv3x3_forward", "conv1x1_wgrad", "bn_backward_from_partials",
                                 "conv1x1_bwd_fused", "bn_moments", "gemm_nt"])
    try:
        lf = F.cross_entropy(fused(x16).float(), y)
        lf.backward()
    finally:
        for n, f in orig.items():
            setattr(C, n, f)
    l32 = F.cross_entropy(ref32(x16.float()), y)
    l32.backward()
    l16 = F.cross_entropy(ref16(x16).float(), y)
    l16.backward()
    _run_three.ref16 = ref16
    # every fused path ran: 1x1 GEMM fwd (36 convs; the deep-K ones (Cin >= 1024) run the LDS-DMA
    # gemm_nt with its statistics epilogue) +
    # stride-1 dgrad (layer-1 conv3 x 3 and the downsample as the fused dgrad+wgrad kernel), 3x3
    # implicit GEMM (16 forward + 12 stride-1 dgrad), MFMA wgrad, EpiLink epilogue + its BN finalize
    assert counts["conv1x1_bwd_fused"] >= 4, counts
    assert (counts["conv1x1_gemm"] + counts["conv1x1_bwd_fused"]
            + counts["bn_moments"] + counts["gemm_nt"] >= 36 + 30), counts
    assert counts["conv3x3_forward"] >= 16 + 12, counts
    assert counts["conv1x1_wgrad"] + counts["conv1x1_bwd_fused"] >= 32, counts
    assert counts.get("epilink", 0) >= 12 and counts["bn_backward_from_partials"] >= 12, counts
    assert abs(lf.item() - l32.item()) < 0.05 * abs(l32.item()) + 0.02, (lf.item(), l32.item(), l16.item())
    sf, s16 = _grad_stats(fused, ref32), _grad_stats(ref16, ref32)
    for grp in ("conv1", "layer1", "layer2", "layer3", "layer4", "fc"):
        rf = sorted(sf[n][0] for n in sf if n.startswith(grp))
        r16 = sorted(s16[n][0] for n in s16 if n.startswith(grp))
        cf = sorted(sf[n][1] for n in sf if n.startswith(grp))
        print(f"\n[gamma={branch_gamma}] {grp:7s} median rel-L2 vs fp32: fused {rf[len(rf) // 2]:.4f}  torch-bf16 "
              f"{r16[len(r16) // 2]:.4f}  min cos fused {cf[0]:.4f}", end="")
    print()
    return fused, ref32, sf, s16


def test_resnet50_bf16_fused_full_model_grads_vs_fp32():
    """Standard (torchvision) init. A random-init BN ResNet amplifies perturbations exponentially
    with depth (mean-field BN gradient explosion), so ANY bf16 stack's gradients are far from fp32
    there — torch's own bf16 ResNet-50 included (median rel-L2 ~1.2 on MI355X). The criterion is
    relative to that yardstick: per parameter and per layer group the fused stack must be as
    accurate as plain bf16 torch."""
    fused, ref32, sf, s16 = _run_three(16, 224)
    for n, (rel, cos) in sf.items():
        assert rel <= 1.5 * s16[n][0] + 0.02, (n, rel, s16[n][0])
    for grp in ("conv1", "layer1", "layer2", "layer3", "layer4", "fc"):
        rf = sorted(sf[n][0] for n in sf if n.startswith(grp))
        r16 = sorted(s16[n][0] for n in s16 if n.startswith(grp))
        assert rf[len(rf) // 2] <= 1.1 * r16[len(r16) // 2] + 0.01, grp
    # BN running statistics: as close to fp32 as torch-bf16's (same yardstick)
    for (n, a), b, c in zip(fused.named_buffers(), ref32.buffers(), _run_three.ref16.buffers()):
        if a.is_floating_point():
            ef, e16 = (a.float() - b).norm().item(), (c.float() - b).norm().item()
            assert ef <= 1.5 * e16 + 1e-3 * (b.norm().item() + 1), (n, ef, e16)


def test_resnet50_bf16_fused_grads_well_conditioned():
    """Residual branches down-weighted (every bn3 gamma = 0.2, SkipInit-style): the same kernels in
    a better-conditioned network (torch-bf16 median rel-L2 vs fp32 drops from ~1.2 to ~0.37 on
    MI355X). Same yardstick criteria, plus direction: per parameter the fused gradient's cosine to
    fp32 is within 0.05 of torch-bf16's."""
    fused, ref32, sf, s16 = _run_three(16, 224, branch_gamma=0.2)
    for n, (rel, cos) in sf.items():
        assert rel <= 1.5 * s16[n][0] + 0.02, (n, rel, s16[n][0])
        assert cos >= s16[n][1] - 0.05, (n, cos, s16[n][1])
    mf = sorted(r for r, _ in sf.values())[len(sf) // 2]
    m16 = sorted(r for r, _ in s16.values())[len(s16) // 2]
    assert mf <= 1.1 * m16 + 0.01, (mf, m16)


def test_resnet50_overfit_curve_tracks_fp32_reference():
    """30 SGD steps on one fixed batch (bs16 @ 224, lr 0.02, momentum 0.9): the xddp stack (DDP
    Reducer + fused kernels + FusedSGD with fp32 master weights) and an fp32 torch model (nn.BN,
    torch SGD) start from identical weights; their loss curves must track each other and both
    must fit the batch."""
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as dist
    from distributeddataparallel_amd.optim import FusedSGD
    from distributeddataparallel_amd.utils.spawn import free_port

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
    try:
        fused, ref32, _, x16, y = _models(16, 224, seed=3)
        ddp = xddp.DDP(fused, device_ids=[0], gradient_as_bucket_view=True)
        o1 = FusedSGD(ddp.parameters(), lr=0.02, momentum=0.9, weight_decay=1e-4, master_weights=True)
        o2 = torch.optim.SGD(ref32.parameters(), lr=0.02, momentum=0.9, weight_decay=1e-4)
        x32 = x16.float()
        la, lb = [], []
        for _ in range(30):
            o1.zero_grad(set_to_none=True)
            loss = F.cross_entropy(ddp(x16).float(), y)
            loss.backward()
            o1.step()
            la.append(loss.item())
            o2.zero_grad(set_to_none=True)
            loss = F.cross_entropy(ref32(x32), y)
            loss.backward()
            o2.step()
            lb.append(loss.item())
        print("\nxddp :", [round(v, 3) for v in la])
        print("fp32 :", [round(v, 3) for v in lb])
        assert abs(la[0] - lb[0]) < 0.05 * lb[0]
        for i in range(10):  # early steps: the same trajectory
            assert abs(la[i] - lb[i]) < 0.1 * lb[0], (i, la[i], lb[i])
        # later steps: lr 0.02 + momentum 0.9 on 16 random labels is a chaotic regime (spikes in
        # the fp32 run too), so trajectories decorrelate; both stacks must fit the batch
        assert min(la) < 0.3 * la[0] and min(lb) < 0.3 * lb[0], (min(la), min(lb))
        assert all(torch.isfinite(torch.tensor(la)))
    finally:
        dist.destroy_process_group()


def test_config3_no_sync_accumulation_bf16_fused_vs_fp32():
    """BASELINE config 3: bf16 channels_last ResNet-50 with FusedBatchNorm2d under the xddp DDP,
    two micro-batches of 16 @ 224 — the first inside ``no_sync()`` (gradients accumulate locally,
    nothing is launched), the second synced (the accumulated gradients go through the bucket copy
    and the all-reduce path). Oracle: an fp32 torch model accumulating the same two backward passes;
    yardstick: the same bf16 model through plain torch ops (SkipInit-conditioned, as above)."""
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as dist
    from distributeddataparallel_amd.utils.spawn import free_port

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
    try:
        fused, ref32, ref16, xa, ya = _models(16, 224, seed=5, branch_gamma=0.2)
        g = torch.Generator(device="cuda").manual_seed(77)
        xb = torch.randn(16, 3, 224, 224, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        yb = torch.randint(0, 1000, (16,), device="cuda", generator=g)
        ddp = xddp.DDP(fused, device_ids=[0], gradient_as_bucket_view=True)
        for it in range(2):  # iteration 0 = one bucket; iteration 1 = the rebuilt layout
            for m in (fused, ref32, ref16):
                m.zero_grad(set_to_none=True)
            launches0 = ddp.reducer.native_launches()
            with ddp.no_sync():
                F.cross_entropy(ddp(xa).float(), ya).backward()
            assert ddp.reducer.native_launches() == launches0, "no_sync must not pack or launch buckets"
            F.cross_entropy(ddp(xb).float(), yb).backward()
            for m, conv in ((ref32, lambda t: t.float()), (ref16, lambda t: t)):
                F.cross_entropy(m(conv(xa)).float(), ya).backward()
                F.cross_entropy(m(conv(xb)).float(), yb).backward()
            torch.cuda.synchronize()
            sf, s16 = _grad_stats(fused, ref32), _grad_stats(ref16, ref32)
            # two bf16 backward passes accumulate into bf16 .grad here (as in torch-bf16): the
            # direction tolerance is 0.08 (the single-step test above uses 0.05)
            for n, (rel, cos) in sf.items():
                assert rel <= 1.5 * s16[n][0] + 0.02, (it, n, rel, s16[n][0])
                assert cos >= s16[n][1] - 0.08, (it, n, cos, s16[n][1])
            mf = sorted(r for r, _ in sf.values())[len(sf) // 2]
            m16 = sorted(r for r, _ in s16.values())[len(s16) // 2]
            assert mf <= 1.1 * m16 + 0.01, (it, mf, m16)
        print(f"\nconfig 3 (no_sync x2): median rel-L2 vs fp32 fused {mf:.4f} torch-bf16 {m16:.4f}")
    finally:
        dist.destroy_process_group()
