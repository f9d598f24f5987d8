#!/usr/bin/env python
"""PMC workload: the 1x1 weight gradient (conv1x1_wgrad) at ResNet-50 layer-2/3/4 shapes, 3 calls each
(profiles/r6_wgrad1x1_ring_ab.txt: the r6 LDS-DMA ring variant measured with it)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_amd._native import load  # noqa: E402

SHAPES = [("l2 conv1", 512, 128, 28, 1), ("l3 conv1", 1024, 256, 14, 1), ("l4 conv1", 2048, 512, 7, 1),
          ("l3 ds", 512, 1024, 14, 2)]
C = load()
g = torch.Generator(device="cuda").manual_seed(0)
cl = torch.channels_last
for label, K, N, H, s in SHAPES:
    dy = torch.randn(256, N, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    x = torch.randn(256, K, H * s, H * s, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.empty(N, K, 1, 1, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        C.conv1x1_wgrad(dy, x, s, w)
    torch.cuda.synchronize()
    print(label, flush=True)
