#!/usr/bin/env python
"""Where do the small copies / fills of a training step come from? Runs the bench's ResNet-50
step (xddp DDP, fused BN, SGD) for a few warmup iterations, then one profiled iteration under
torch.profiler with Python stacks, and prints every aten::copy_ / fill_ / zero_ / clone /
contiguous call with its count, device time and the innermost frames of this repository that
issued it.

usage: python scripts/step_ops.py [--batch-size 256] [--out FILE]
"""
import argparse
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=256)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd import models
    from distributeddataparallel_amd.optim import FusedSGD

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    xdist.init_process_group("nccl", rank=0, world_size=1)
    torch.cuda.set_device(0)
    from distributeddataparallel_amd.ops.batch_norm import FusedBatchNorm2d

    m = models.resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    ddp = xddp.DDP(m, device_ids=[0], gradient_as_bucket_view=True)
    opt = FusedSGD(ddp.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4, master_weights=True)
    x = torch.randn(a.batch_size, 3, 224, 224, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch_size,), device="cuda")

    def step():
        opt.zero_grad(set_to_none=True)
        F.cross_entropy(ddp(x).float(), y).backward()
        opt.step()

    for _ in range(4):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    want = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::clone", "aten::contiguous", "aten::zeros",
            "aten::zeros_like", "aten::empty_like", "aten::to", "aten::_to_copy")
    agg = defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.name not in want:
            continue
        frames = [f for f in (ev.stack or []) if "distributeddataparallel_amd" in f or "step_ops.py" in f][:3]
        key = (ev.name, " <- ".join(frames) or "(no repo frame)")
        agg[key][0] += 1
        agg[key][1] += ev.device_time_total
    lines = [f"# one ResNet-50 bs{a.batch_size} xddp step: copy / fill ops by issuing site (count, device us)"]
    for (name, where), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{n:4d} {us:9.1f} us  {name:18s} {where}")
    kern = defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and ("copyBuffer" in ev.name or "fillBuffer" in ev.name):
            kern[ev.name][0] += 1
            kern[ev.name][1] += ev.device_time_total
    lines.append("# runtime copy / fill kernels in the step")
    for k, (n, us) in kern.items():
        lines.append(f"{n:4d} {us:9.1f} us  {k}")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    xdist.destroy_process_group()


if __name__ == "__main__":
    main()
