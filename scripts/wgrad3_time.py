#!/usr/bin/env python
"""3x3 weight-gradient kernel per call at the ResNet-50 bs256 stride-1 shapes, with the variant
environment switches given as arguments (NAME=VALUE ...) A/B'd in one process.

usage: python scripts/wgrad3_time.py [--iters 20] [VAR=VAL,VAR=VAL ...]
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
    ap.add_argument("--splits", default="0", help="comma list of pixel splits per tile (0 = the default)")
    ap.add_argument("--only", type=int, default=-1, help="run only this shape index")
    ap.add_argument("variants", nargs="*", default=[""])
    a = ap.parse_args()
    C = load()
    g = torch.Generator(device="cuda").manual_seed(3)
    shapes = [(64, 56, 64, 1), (128, 28, 128, 1), (256, 14, 256, 1), (512, 7, 512, 1), (128, 56, 128, 2),
              (256, 28, 256, 2), (512, 14, 512, 2)]
    if a.only >= 0:
        shapes = [shapes[a.only]]
    for c, hw, n, st in shapes:
        x = torch.randn(256, c, hw, hw, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        oh = (hw - 1) // st + 1
        dy = torch.randn(256, n, oh, oh, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = torch.empty(n, c, 3, 3, device="cuda", dtype=torch.bfloat16)
        ref = None
        for var in [(v, int(sp)) for v in a.variants for sp in a.splits.split(",")]:
            var, sp = var
            saved = {}
            for kv in filter(None, var.split(",")):
                k, v = kv.split("=", 1)
                saved[k] = os.environ.get(k)
                os.environ[k] = v
            out = C.conv3x3_wgrad_patch(dy, x, st, w, sp).float()
            if ref is None:
                ref = out
            err = ((out - ref).norm() / ref.norm()).item()
            for _ in range(3):
                C.conv3x3_wgrad_patch(dy, x, st, w, sp)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.iters):
                C.conv3x3_wgrad_patch(dy, x, st, w, sp)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / a.iters * 1e3
            flops = 2.0 * 256 * oh * oh * n * c * 9
            print(json.dumps({"shape": f"C{c} {hw}x{hw} N{n} s{st}", "variant": var or "default", "splits": sp, "us": round(us, 1),
                              "tflops": round(flops / us / 1e6, 1), "rel_vs_first": round(err, 6)}), flush=True)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v


if __name__ == "__main__":
    main()
