#!/usr/bin/env python
"""Per-call time of the stride-1 3x3 conv kernels at the ResNet-50 bs256 shapes: the dispatcher's
path (conv3x3_forward: row-band kernel or dense-GEMM path) and the row-band kernel called directly
(conv3x3_band_forward, optional band heights and configurations), forward with BN statistics and
the input gradient (no statistics), plus the weight gradient; us per call and TF/s.

usage: python scripts/c3_time.py [--iters 20] [--rows 56:4,28:7,...] [--batch 256]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):  # best of three back-to-back batches
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
    ap.add_argument("--rows", default="", help="W:R,... band heights for the direct band calls")
    ap.add_argument("--cfgs", default="-1", help="comma list of band kernel configurations to time")
    ap.add_argument("--wgrad-only", action="store_true", help="time the weight gradient only (stride 1 and 2)")
    a = ap.parse_args()
    C = load()
    rows = {int(k): int(v) for k, v in (p.split(":") for p in a.rows.split(",") if p)}
    g = torch.Generator(device="cuda").manual_seed(0)
    if a.wgrad_only:
        for c, hw, st in ((64, 56, 1), (128, 28, 1), (256, 14, 1), (512, 7, 1), (128, 56, 2), (256, 28, 2), (512, 14, 2)):
            x = torch.randn(a.batch, c, hw, hw, device="cuda", generator=g).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            oh = (hw - 1) // st + 1
            dy = torch.randn(a.batch, c, oh, oh, device="cuda", generator=g).to(torch.bfloat16).contiguous(
                memory_format=torch.channels_last)
            w = torch.empty(c, c, 3, 3, device="cuda", dtype=torch.bfloat16)
            t = timed(lambda: C.conv3x3_wgrad_patch(dy, x, st, w), a.iters)
            fl = 2.0 * a.batch * oh * oh * c * 9 * c
            print(f"wgrad C{c} {hw}x{hw} s{st}: {t:7.1f} us {fl / t / 1e6:6.0f} TF/s", flush=True)
        return
    cfgs = [int(c) for c in a.cfgs.split(",")]
    print(f"{'shape':18s} {'path fwd':>14s} {'path dgrad':>14s} {'wgrad':>14s} " +
          " ".join(f"{'band%d fwd' % c:>14s} {'band%d dgrad' % c:>14s}" for c in cfgs))
    for c, hw in ((64, 56), (128, 28), (256, 14), (512, 7)):
        B = a.batch
        x = torch.randn(B, c, hw, hw, device="cuda", generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device="cuda", generator=g) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        rot = C.conv3x3_rot_weight(w)
        fl = 2.0 * B * hw * hw * c * 9 * c
        r = rows.get(hw, 0)
        res = [timed(lambda: C.conv3x3_forward(x, w, 1, True), a.iters),
               timed(lambda: C.conv3x3_forward(x, rot, 1, False), a.iters),
               timed(lambda: C.conv3x3_wgrad_patch(x, x, 1, w), a.iters)]
        err = 0.0
        y0 = C.conv3x3_forward(x, w, 1, False)[0].float()
        for cf in cfgs:
            try:
                y1 = C.conv3x3_band_forward(x, w, False, r, cf)[0].float()
            except RuntimeError:  # configuration does not cover this shape
                res += [float("nan"), float("nan")]
                continue
            res += [timed(lambda: C.conv3x3_band_forward(x, w, True, r, cf), a.iters),
                    timed(lambda: C.conv3x3_band_forward(x, rot, False, r, cf), a.iters)]
            # the band kernel agrees with the dispatcher's path
            err = max(err, (y0 - y1).abs().max().item() / max(1e-6, y0.abs().max().item()))
        cols = " ".join(f"{t:7.1f}us {fl / t / 1e6:5.0f}" for t in res)
        print(f"C{c:<4d} {hw}x{hw:<3d} N{c:<4d} {cols}  relerr {err:.1e}", flush=True)


if __name__ == "__main__":
    main()
