#!/usr/bin/env python
"""PMC workload: the stride-1 3x3 kernels at the ResNet-50 bs256 shapes, 3 calls each (dispatcher
path forward + statistics, its input gradient, the row-band kernel forward / input gradient, the
weight gradient). Run under rocprofv3 --pmc ...; summarize with scripts/pmc_group.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
for c, hw in ((64, 56), (128, 28), (256, 14), (512, 7)):
    if only and str(hw) not in only:
        continue
    x = torch.randn(256, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    rot = C.conv3x3_rot_weight(w)
    for fn in (lambda: C.conv3x3_forward(x, w, 1, True), lambda: C.conv3x3_forward(x, rot, 1, False),
               lambda: C.conv3x3_band_forward(x, w, True, 0, -1), lambda: C.conv3x3_band_forward(x, rot, False, 0, -1),
               lambda: C.conv3x3_wgrad_patch(x, x, 1, w)):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
print("c3_pmc done")
