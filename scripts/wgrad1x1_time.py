#!/usr/bin/env python
"""1x1 convolution weight gradient (conv1x1_wgrad: dW = dYᵀ·X over the pixel dimension, fp32 split
partials + reduce) per call at every ResNet-50 bs256 1x1 shape, with its HBM floor (dY + X bytes at
5.5 TB/s) and MFMA floor (2.2 PF/s) and hipBLASLt's time for dYᵀ·X at stride 1, so the distance to the roofline is visible per shape.

usage: python scripts/wgrad1x1_time.py [--iters 20] [--batch 256]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_amd._native import load  # noqa: E402

# (label, K = input channels, N = output channels, output H, stride)
SHAPES = [
    ("l1 conv1 b1", 64, 64, 56, 1), ("l1 conv1", 256, 64, 56, 1), ("l1 conv3", 64, 256, 56, 1),
    ("l2 conv1 b1", 256, 128, 56, 1), ("l2 conv1", 512, 128, 28, 1), ("l2 conv3", 128, 512, 28, 1),
    ("l2 ds", 256, 512, 28, 2),
    ("l3 conv1 b1", 512, 256, 28, 1), ("l3 conv1", 1024, 256, 14, 1), ("l3 conv3", 256, 1024, 14, 1),
    ("l3 ds", 512, 1024, 14, 2),
    ("l4 conv1 b1", 1024, 512, 14, 1), ("l4 conv1", 2048, 512, 7, 1), ("l4 conv3", 512, 2048, 7, 1),
    ("l4 ds", 1024, 2048, 7, 2),
]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    C = load()
    g = torch.Generator(device="cuda").manual_seed(0)
    cl = torch.channels_last
    for label, K, N, H, s in SHAPES:
        B = a.batch
        dy = torch.randn(B, N, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
        x = torch.randn(B, K, H * s, H * s, device="cuda", generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
        w = torch.empty(N, K, 1, 1, device="cuda", dtype=torch.bfloat16)
        t = timed(lambda: C.conv1x1_wgrad(dy, x, s, w), a.iters)
        M = B * H * H
        tl = float("nan")
        if s == 1:  # hipBLASLt on the same operands: dW = dY[M, N]ᵀ · X[M, K]
            d2, x2 = dy.permute(0, 2, 3, 1).reshape(M, N), x.permute(0, 2, 3, 1).reshape(M, K)
            tl = timed(lambda: torch.mm(d2.t(), x2), a.iters)
        fl = 2.0 * M * N * K
        by = 2.0 * (dy.numel() + M * K)  # (strided: only the sampled input pixels are read)
        print(json.dumps({"shape": f"{label} M{M} K{K} N{N} s{s}", "us": round(t, 1),
                          "tflops": round(fl / t / 1e6, 1), "TBps": round(by / t / 1e6, 2),
                          "floor_us": round(max(by / 5.5e6, fl / 2.2e9), 1), "hipblaslt_us": round(tl, 1)}), flush=True)


if __name__ == "__main__":
    main()
