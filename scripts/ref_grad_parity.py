#!/usr/bin/env python
"""fp32 gradient parity of the reference model (ResNet-18, 10 classes, 32x32, batch 32) between
the xddp stack (FusedBatchNorm2d, channels_last, MIOpen convs) and torch's (nn.BatchNorm2d, NCHW),
with an fp64 CPU model as ground truth: per-parameter max relative gradient error of each."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_amd.models import SimpleCNN  # noqa: E402
from distributeddataparallel_amd.ops import FusedBatchNorm2d  # noqa: E402


def grads(model, x, y):
    model.zero_grad()
    F.cross_entropy(model(x), y).backward()
    return {n: p.grad.detach().double().cpu() for n, p in model.named_parameters()}


def main():
    torch.manual_seed(0)
    ref = SimpleCNN().double()
    sd = ref.state_dict()
    x = torch.randn(32, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (32,))
    g64 = grads(ref, x, y)
    tm = SimpleCNN().cuda()
    tm.load_state_dict(sd)
    xm = SimpleCNN(norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last)
    xm.load_state_dict(sd)
    for flag in (True, False):
        torch.backends.cudnn.allow_tf32 = flag
        gt = grads(tm, x.float().cuda(), y.cuda())
        gx = grads(xm, x.float().cuda().contiguous(memory_format=torch.channels_last), y.cuda())
        print(f"== cudnn.allow_tf32={flag}")
        worst_t = worst_x = 0.0
        for n in g64:
            s = g64[n].abs().max().item() + 1e-30
            et = (gt[n] - g64[n]).abs().max().item() / s
            ex = (gx[n] - g64[n]).abs().max().item() / s
            worst_t, worst_x = max(worst_t, et), max(worst_x, ex)
            if ex > 1e-3 or et > 1e-3:
                print(f"{n:40s} torch {et:.2e}  xddp {ex:.2e}")
        print(f"worst rel err: torch {worst_t:.2e}  xddp {worst_x:.2e}")


if __name__ == "__main__":
    main()
