#!/usr/bin/env python
"""Register-staged 1x1 GEMM (conv1x1_gemm) per call at the ResNet-50 bs256 bottleneck conv3 shapes,
plain / + BN statistics / + BN-apply prologue / + the prologue's side output (the pending-apply
form the model runs), so the cost of each fused piece is visible.

usage: python scripts/gemm1x1_time.py [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_amd._native import load  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", type=int, default=-1, help="run only this shape index")
    a = ap.parse_args()
    C = load()
    g = torch.Generator(device="cuda").manual_seed(5)
    # (K, N, H): conv3 of layer1..4 (planes -> 4 planes)
    shapes = [(64, 256, 56), (128, 512, 28), (256, 1024, 14), (512, 2048, 7)]
    for K, N, H in (shapes if a.only < 0 else [shapes[a.only]]):
        x = torch.randn(256, K, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(N, K, 1, 1, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        ss = torch.cat([torch.rand(K, device="cuda", generator=g) + 0.5,
                        torch.randn(K, device="cuda", generator=g) * 0.1]).contiguous()
        out = torch.empty_like(x)
        variants = {
            "plain": lambda: C.conv1x1_gemm(x, w, 1, None, False),
            "stats": lambda: C.conv1x1_gemm(x, w, 1, None, True),
            "pro1+stats": lambda: C.conv1x1_gemm(x, w, 1, ss, True),
            "pro1+stats+side": lambda: C.conv1x1_gemm(x, w, 1, ss, True, pro_out=out),
        }
        for name, fn in variants.items():
            for _ in range(3):
                fn()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.iters):
                fn()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.iters * 1e3
            M = 256 * H * H
            print(json.dumps({"shape": f"M{M} K{K} N{N}", "variant": name, "us": round(us, 1),
                              "tflops": round(2.0 * M * K * N / us / 1e6, 1)}), flush=True)




def epi_main():
    """--epi: the input-gradient GEMM with the BN-reduce epilogue (EPI, form 1: + identity gradient,
    ReLU mask bits, BN-backward partials) at the bottleneck conv1 shapes."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--epi", action="store_true")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", type=int, default=-1)
    a = ap.parse_args()
    C = load()
    g = torch.Generator(device="cuda").manual_seed(6)
    # (planes K, in/out channels N, H)
    shapes = [(64, 256, 56), (128, 512, 28), (256, 1024, 14), (512, 2048, 7)]
    for K, N, H in (shapes if a.only < 0 else [shapes[a.only]]):
        bf = dict(device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(256, K, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(K, N, 1, 1, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
        add = torch.randn(256, N, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        y = torch.randn(256, N, H, H, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        bits = torch.randint(0, 255, (y.numel() // 8,), device="cuda", dtype=torch.uint8, generator=g)
        mean = torch.randn(N, device="cuda", generator=g)
        del bf

        def fn():
            return C.conv1x1_gemm(dy, w, 1, None, False, None, True, add, y, bits, mean, None, 1)

        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        M = 256 * H * H
        gb = (M * K + 3 * M * N) * 2 / 1e9 + M * N / 8 / 1e9
        print(json.dumps({"shape": f"EPI M{M} K{K} N{N}", "us": round(us, 1), "TBps": round(gb / us * 1e3, 2),
                          "tflops": round(2.0 * M * K * N / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    epi_main() if "--epi" in sys.argv else main()
