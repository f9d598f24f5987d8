#!/usr/bin/env python
"""Two-shot peer all-reduce under concurrent compute: W processes share cuda:0, each runs a chain
of bf16 GEMMs on its default stream while bucket-sized two-shot all-reduces (the ResNet-50 bucket
sizes) run on a side stream, started as each "bucket" becomes ready — the DDP backward pattern.

usage: python scripts/peer_stress.py [--world 2] [--iters 5] [--priority high|normal]
                                     [--compute 1|0] [--blocks N] [--timeout-ms 20000]
Prints one line per iteration and per rank; a peer that never arrives surfaces as status=1 after
--timeout-ms (the kernels then drain), never as a hang.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

SIZES = [2049008, 14438400, 9069632]  # bf16 elements of the ResNet-50 buckets (reference policy)


def _rank(rank, world, a):
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd._native import load

    C = load()
    torch.cuda.set_device(0)
    pg = xdist.get_default_group()
    peer = C.PeerAllReduce(C.PrefixStore("stress", pg.store), rank, world, 0, 1 << 20, 64 << 20, a.timeout_ms / 1e3)
    side = torch.cuda.Stream(priority=-1 if a.priority == "high" else 0)
    bufs = [torch.full((n,), float(rank + 1), device="cuda", dtype=torch.bfloat16) for n in SIZES]
    m = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    total = float(sum(range(1, world + 1)))
    torch.cuda.synchronize()
    for it in range(a.iters):
        for b in bufs:
            b.fill_(float(rank + 1))
        t0 = time.time()
        x = m
        for b in bufs:
            if a.compute:
                for _ in range(6):  # ~0.1 ms each: the "backward" between bucket-ready points
                    x = torch.mm(x, m) * 1e-3
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(side):
                side.wait_event(ev)
                peer.allreduce_two_shot(b, 0)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        ok = all(torch.all(b.float() == total).item() for b in bufs)
        print(f"[stress] rank {rank} iter {it}: {1e3 * (time.time() - t0):.1f} ms status={peer.status()} ok={ok}",
              flush=True)
        if peer.status() != 0 or not ok:
            raise SystemExit(f"rank {rank}: two-shot failed at iter {it}")
    xdist.barrier()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--priority", choices=["high", "normal"], default="high")
    ap.add_argument("--compute", type=int, default=1)
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--timeout-ms", type=float, default=20000.0)
    a = ap.parse_args()
    if a.blocks:
        os.environ["XDDP_PEER_TWO_SHOT_BLOCKS"] = str(a.blocks)
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
    from _dist_utils import run_ranks

    print(f"[stress] world={a.world} priority={a.priority} compute={a.compute} blocks={a.blocks or 64}", flush=True)
    run_ranks(_rank, world=a.world, args=(a,))
    print("[stress] ok", flush=True)


if __name__ == "__main__":
    main()
