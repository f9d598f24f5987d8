#!/usr/bin/env python
"""Does the overlapped optimizer hide the tail all-reduce? Reads a rocprofv3 kernel trace of
``bench.py --overlap-optim 1`` (forced RCCL launches at W=1: XDDP_RCCL_FORCE_LAUNCH=1, so every
bucket's all-reduce is a real RCCL kernel on the comm stream) and reports, per iteration, the
tail window — the LAST ``--tail-chunks`` all-reduce kernels (the tail bucket, all-reduced in that
many chunks by the "tail" schedule; 1 for the "backward" schedule) — and the AdamW update kernels
that ran while it was in flight, plus how much of the AdamW time overlapped any all-reduce at all.

usage: python scripts/overlap_trace.py TRACE_DIR [--tail-chunks K] [--out FILE]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default=None)
    ap.add_argument("--tail-chunks", type=int, default=1)
    a = ap.parse_args()
    f = sorted(glob.glob(os.path.join(a.trace, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    ar = [(s, e) for s, e, n in ev if "oneRankReduce" in n or "ncclDevKernel" in n]
    adam = [(s, e) for s, e, n in ev if "adam_kernel" in n]
    # iterations: all-reduces separated by more than 20 ms (between two backward passes there is
    # a forward and the loss; inside a backward the buckets follow each other within a few ms)
    lines = [f"# {os.path.basename(f)}: {len(ar)} all-reduce kernels, {len(adam)} AdamW update kernels"]
    if not ar:
        text = "\n".join(lines + ["no all-reduce kernels in the trace"]) + "\n"
        print(text)
        return
    iters, cur = [], [ar[0]]
    for p, q in zip(ar, ar[1:]):
        if q[0] - p[1] > 20_000_000:
            iters.append(cur)
            cur = []
        cur.append(q)
    iters.append(cur)
    tot_adam = sum(e - s for s, e in adam)

    def overlap(x, ys):
        return sum(max(0, min(x[1], e) - max(x[0], s)) for s, e in ys)

    lines.append(f"tail window = the last {a.tail_chunks} all-reduce kernel(s) of each iteration")
    lines.append(f"{'iter':>4s} {'allreduces':>10s} {'tail ms':>8s} {'AdamW kernels during tail':>26s} "
                 f"{'AdamW ms under tail':>20s} {'AdamW before tail start':>24s} {'AdamW after tail end':>21s} "
                 f"{'last AdamW end - tail end ms':>29s}")
    for i, it in enumerate(iters):
        k = min(len(it), a.tail_chunks)
        tail = (it[-k][0], it[-1][1])
        during = [x for x in adam if x[0] < tail[1] and x[1] > tail[0]]
        before = [x for x in adam if x[1] <= tail[0] and x[0] >= it[0][0]]
        nxt = iters[i + 1][0][0] if i + 1 < len(iters) else float("inf")
        after = [x for x in adam if x[0] >= tail[1] and x[1] <= nxt]
        last = max((x[1] for x in after), default=tail[1])
        lines.append(f"{i:4d} {len(it):10d} {(tail[1] - tail[0]) / 1e6:8.3f} {len(during):26d} "
                     f"{overlap(tail, adam) / 1e6:20.3f} {len(before):24d} {len(after):21d} "
                     f"{(last - tail[1]) / 1e6:29.3f}")
    under_any = sum(overlap(x, ar) for x in adam)
    lines.append(f"AdamW kernel time {tot_adam / 1e6:.3f} ms, of which {under_any / 1e6:.3f} ms ran while an "
                 f"all-reduce kernel was executing")
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main()
