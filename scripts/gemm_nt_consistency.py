#!/usr/bin/env python
"""Why did r5's two artifacts disagree on ViT fc1 (own gemm_nt 0.87x of hipBLASLt in
r5_gemm_nt_vs_hipblaslt.txt, 0.57x in r5_pmc_kernels_final.txt)? VERDICT r5 "Next round" #8.

The sweep (scripts/gemm_nt_bench.py) times 20 back-to-back calls with events after warm-up, fc1
right after the ViT qkv / proj shapes. The PMC workload (scripts/pmc_r3.py) runs 3 calls per op,
fc1 right after the 8192^3 own / hipBLASLt blocks (~2.4 ms of sustained full-chip MFMA load).
This script times fc1 (own and hipBLASLt) in both contexts and in both orders, 3 and 20 calls,
each call bracketed by its own events, so the per-call times show whether the first calls after
a heavy block run slow (clock / power recovery) or whether the op itself differs.

usage: python scripts/gemm_nt_consistency.py   (one JSON line per context)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
M, K, N = 12608, 1024, 4096


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16).contiguous()


def per_call(fn, calls):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(calls)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return [round(s.elapsed_time(e) * 1e3, 1) for s, e in ev]


def heavy():
    """the PMC workload's preceding block: 8192^3 own + hipBLASLt, 4 calls each"""
    a, w = bf(8192, 8192), bf(8192, 8192, scale=8192 ** -0.5)
    for _ in range(4):
        C.gemm_nt(a, w)
    for _ in range(4):
        torch.mm(a, w.t())
    del a, w


def main():
    a, w = bf(M, K), bf(N, K, scale=K ** -0.5)
    own = lambda: C.gemm_nt(a, w)  # noqa: E731
    blas = lambda: torch.mm(a, w.t())  # noqa: E731
    own()
    blas()
    torch.cuda.synchronize()
    fl = 2.0 * M * N * K
    for ctx in ("idle", "after_8192_block"):
        for first, calls in (("own", 3), ("blas", 3), ("own", 20), ("blas", 20)):
            for name, fn in ((first, own if first == "own" else blas),):
                if ctx == "after_8192_block":
                    heavy()
                else:
                    torch.cuda.synchronize()
                    torch.cuda._sleep(50_000_000)  # ~idle gap before the op
                    torch.cuda.synchronize()
                us = per_call(fn, calls)
                steady = sorted(us)[len(us) // 2]
                print(json.dumps({"context": ctx, "op": name, "calls": calls, "per_call_us": us,
                                  "median_us": steady, "median_tflops": round(fl / steady / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
