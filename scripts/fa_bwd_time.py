#!/usr/bin/env python
"""Flash-attention backward (own HIP kernels) per call at the BASELINE transformer shapes:
Llama-3-8B (B2 S4096 H32/8 D128 causal, the PMC table's shape) and ViT-L/16 (B256 S197 H16 D64).
Prints analytic TF/s (5 GEMMs of the backward with one recompute; causal counts half), so
variants selected by environment switches can be A/B'd in one box.

usage: python scripts/fa_bwd_time.py [--iters 20] [--bias]
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
    ap.add_argument("--bias", action="store_true", help="ViT: also return the qkv bias gradient (bias_like)")
    a = ap.parse_args()
    C = load()
    for name, B, S, H, Hkv, D, causal in (("llama", 2, 4096, 32, 8, 128, True), ("vit", 256, 197, 16, 16, 64, False)):
        g = torch.Generator(device="cuda").manual_seed(0)
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, generator=g)
        v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, generator=g)
        do = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, generator=g)
        scale = D ** -0.5
        o, lse = C.flash_attn_forward(q, k, v, causal, scale)
        bl = torch.zeros(3 * H * D, device="cuda", dtype=torch.bfloat16) if a.bias and name == "vit" else None
        run = lambda: C.flash_attn_backward(do, q, k, v, o, lse, causal, scale, None, None, None, bl)  # noqa: E731
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        flops = 5 * 2.0 * B * H * S * S * D * (0.5 if causal else 1.0)
        dq, dk, dv = run()[:3]
        print(json.dumps({"shape": name, "bwd_us": round(us, 1), "tflops": round(flops / us / 1e6, 1),
                          "finite": bool(torch.isfinite(dq).all() and torch.isfinite(dk).all())}), flush=True)


if __name__ == "__main__":
    main()
