#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace: per-category ms/step and RCCL/compute overlap.

usage: python scripts/prof_summary.py <prof_kernel_trace.csv> --steps N [--csv-out path]
"""
import argparse
import csv
import re
from collections import defaultdict

CATS = [
    ("RCCL", r"(ncclDevKernel|oneRankReduce|rccl|nccl)"),
    ("xddp 1x1-conv GEMM", r"conv1x1_gemm_kernel"),
    ("xddp 1x1-conv wgrad", r"(conv1x1_wgrad_kernel|wgrad_reduce_kernel)"),
    ("xddp 3x3 conv", r"conv3x3_"),
    ("xddp stem/strided conv", r"(conv_stem|conv_s2|stem_)"),
    ("xddp BN backward", r"bn_bwd_(reduce|elem)"),
    ("xddp BN finalize", r"(finalize_kernel|bn_partial_finalize)"),
    ("xddp BN forward", r"(bn_apply|bn_stats|bn_fwd)"),
    ("xddp max-pool", r"maxpool"),
    ("xddp optimizer/bucket", r"(sgd_|adamw_|scale_copy|copy_bytes|sumsq|nonfinite|mt_)"),
    ("MIOpen conv", r"(igemm_|MIOpen|miopen|naive_conv|gridwise|ck::|device_conv)"),
    ("MIOpen aux", r"(SubTensorOp|Op2dTensor|Op1dTensor|fill|transpose_NCHW|batched_transpose)"),
    ("copies", r"(copyBuffer|direct_copy|elementwise_kernel.*copy)"),
]


def cat(name):
    for c, pat in CATS:
        if re.search(pat, name):
            return c
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, required=True)
    ap.add_argument("--last-fraction", type=float, default=1.0,
                    help="only the last fraction of dispatches (skip warmup)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.last_fraction < 1.0:
        rows = rows[int(len(rows) * (1 - a.last_fraction)):]
    tot = defaultdict(float)
    cnt = defaultdict(int)
    comm, comp = [], []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        c = cat(r["Kernel_Name"])
        tot[c] += (e - s) / 1e6
        cnt[c] += 1
        (comm if c == "RCCL" else comp).append((s, e, r.get("Queue_Id"), r.get("Stream_Id")))
    allt = sum(tot.values())
    print(f"{'category':32s} {'ms/step':>9s} {'share':>7s} {'calls/step':>10s}")
    for c, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{c:32s} {v / a.steps:9.3f} {100 * v / allt:6.1f}% {cnt[c] / a.steps:10.1f}")
    print(f"{'total kernel time':32s} {allt / a.steps:9.3f}")
    if comm:
        # fraction of RCCL kernel time during which some compute kernel was also running
        comp.sort()
        ov = 0
        j = 0
        for s, e, _, _ in comm:
            for cs, ce, _, _ in comp:
                if ce <= s:
                    continue
                if cs >= e:
                    break
                ov += min(e, ce) - max(s, cs)
        ct = sum(e - s for s, e, _, _ in comm)
        qs = sorted({(q, st) for _, _, q, st in comm})
        print(f"RCCL kernels: {len(comm)} ({len(comm) / a.steps:.1f}/step), {ct / 1e6 / a.steps:.3f} ms/step, "
              f"queues/streams {qs}; concurrent with compute kernels for {100 * min(ov, ct) / max(ct, 1):.1f}% of their time")


if __name__ == "__main__":
    main()
