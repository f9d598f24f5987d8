"""Stride-2 3x3 input gradient (conv3x3.hip DG2 phase grids) vs MIOpen, per ResNet-50 shape and
tile config (XDDP_DG2_TILE). Usage: python scripts/dg2_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_amd._native import load  # noqa: E402

C = load()


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


cl = torch.channels_last
for b, c, h in [(256, 128, 56), (256, 256, 28), (256, 512, 14)]:
    x = torch.randn(b, c, h, h, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    oh = (h - 1) // 2 + 1
    dy = torch.randn(b, c, oh, oh, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
    rot = C.conv3x3_rot_weight(w)
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1,
                                              [True, False, False])[0]
    t_mi = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0],
                                                              1, [True, False, False]))
    flops = 2 * b * h * h * c * c * 9 / 4
    line = f"C{c} {h}x{h} bs{b}: MIOpen {t_mi:7.1f} us"
    for cfg in (0, 1, 4, 5):
        os.environ["XDDP_DG2_TILE"] = str(cfg)
        out = C.conv3x3_dgrad_s2(dy, rot, h, h)
        err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
        t = timeit(lambda: C.conv3x3_dgrad_s2(dy, rot, h, h))
        line += f" | tile{cfg} {t:7.1f} us ({flops / t / 1e6:5.0f} TF/s, rel err {err:.1e})"
    print(line, flush=True)
