#!/usr/bin/env python
"""Stride-2 3x3 backward of ResNet-50 (bs256): own kernels vs MIOpen, per shape.

dgrad: conv3x3_dgrad_s2 (gemm.hip DGS2: four phase GEMMs, no zero-fill) vs
aten.convolution_backward(output_mask=[True, False, False]); wgrad: conv3x3_wgrad_patch(stride 2)
vs aten.convolution_backward(output_mask=[False, True, False]). Prints one line per shape and the
max |own - MIOpen| relative to max |MIOpen|.

usage: python scripts/s2_bwd_bench.py [--batch 256] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_amd._native import load  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    C = load()
    cl = torch.channels_last
    torch.backends.cudnn.benchmark = False
    rows = []
    for c, h in ((128, 56), (256, 28), (512, 14)):
        x = torch.randn(a.batch, c, h, h, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        w = (torch.randn(c, c, 3, 3, device="cuda") / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        dy = torch.randn(a.batch, c, h // 2, h // 2, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=cl)
        flops = 2.0 * a.batch * (h // 2) ** 2 * c * c * 9

        def mi(mask):
            return torch.ops.aten.convolution_backward(dy, x, w, None, [2, 2], [1, 1], [1, 1], False, [0, 0], 1, mask)

        wr = C.conv3x3_rot_weight(w)
        t_md = timeit(lambda: mi([True, False, False]), a.iters)
        t_od = timeit(lambda: C.conv3x3_dgrad_s2(dy, wr, h, h), a.iters)
        t_rot = timeit(lambda: C.conv3x3_rot_weight(w), a.iters)
        t_mw = timeit(lambda: mi([False, True, False]), a.iters)
        t_ow = timeit(lambda: C.conv3x3_wgrad_patch(dy, x, 2, w), a.iters)
        ref_dx = mi([True, False, False])[0].float()
        ref_dw = mi([False, True, False])[1].float()
        e_dx = ((C.conv3x3_dgrad_s2(dy, wr, h, h).float() - ref_dx).abs().max() / ref_dx.abs().max()).item()
        e_dw = ((C.conv3x3_wgrad_patch(dy, x, 2, w).float() - ref_dw).abs().max() / ref_dw.abs().max()).item()
        r = {"C": c, "H": h, "dgrad_miopen_us": round(t_md, 1), "dgrad_own_us": round(t_od, 1),
             "rot_weight_us": round(t_rot, 1), "dgrad_own_tflops": round(flops / t_od / 1e6, 1),
             "wgrad_miopen_us": round(t_mw, 1), "wgrad_own_us": round(t_ow, 1),
             "wgrad_own_tflops": round(flops / t_ow / 1e6, 1), "dgrad_rel_err": round(e_dx, 5),
             "wgrad_rel_err": round(e_dw, 5)}
        rows.append(r)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
