"""Init-time calibration of the xGMI communication policy.

The bucket policy (``parallel/bucket_policy.py``) prices one all-reduce of S bytes over W ranks
as ``t(S) = alpha + 2 (W-1)/W * S / B``, and the RCCL communicator can route a message to its own
peer-memory kernels (one-shot / two-shot over IPC-mapped buffers, ``comm/peer_allreduce.hip``)
instead of the RCCL ring. Before this module, alpha / B were assumed constants and the peer route
a manual switch. ``calibrate(pg, sizes)`` measures them on the job's own communicator, once, at
init (outside any timed region):

1. **Self-check of the peer path** (``XDDP_PEER_ALLREDUCE=auto`` creates the lanes on probation:
   nothing is routed to them and their timeouts are not communicator errors). Eight back-to-back
   two-shot all-reduces (plus one-shot ones) of rank-distinct integer patterns whose exact sums
   every rank knows, alternating fp32 / bf16 and message sizes so both staging slots and several
   chunkings are exercised, under a short device-side timeout. Every rank's verdict is combined
   with a MAX all-reduce over the base path: ONE failing rank (wrong data, timeout, missing lane)
   makes every rank close its lanes and keep RCCL, and the reason is reported. On the ``peer``
   backend the base path is the one-shot lane itself, so a failed self-check raises on every rank
   (there is no path left to fall back to); lanes armed without probation
   (``XDDP_PEER_ALLREDUCE=1/2``) get the same data self-check under their configured timeout, and a
   wrong result raises on every rank (nothing to fall back to without ending the communicator).
2. **Timings.** Each route is timed at each probe size (2 warm-up + ``iters`` back-to-back calls,
   host clock around a device sync, so the launch cost is part of alpha); the timing matrix is
   MAX-reduced, so every rank holds identical numbers.
3. **Fit.** alpha and B from the base path's timings (:func:`fit_alpha_busbw`), installed as the
   bucket policy's calibration (:func:`bucket_policy.set_calibration`).
4. **Routes.** Per probe size the fastest route; consecutive sizes with the same winner form one
   segment, segment boundaries are the geometric means of neighbouring probe sizes
   (:func:`choose_routes`). The table goes to the communicator (``set_route_table``); every rank
   computes it from the same MAX-reduced numbers, so every rank routes every message the same way.

All arithmetic on the measured numbers is plain Python on identical inputs: deterministic and the
same on every rank. CPU tests drive :func:`fit_alpha_busbw` / :func:`choose_routes` on synthetic
timings; ``tests/test_calibrate_gpu.py`` runs the whole procedure with two processes on one GPU
over the ``peer`` backend, including a corrupted self-check that must raise on both ranks, and the
RCCL communicator's probation path (fallback to the ring) with forced launches on one rank.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch

ROUTE_AUTO, ROUTE_BASE, ROUTE_ONE_SHOT, ROUTE_TWO_SHOT = 0, 1, 2, 3
ROUTE_NAMES = {ROUTE_BASE: "base", ROUTE_ONE_SHOT: "one_shot", ROUTE_TWO_SHOT: "two_shot"}
_MAX_BOUND = 1 << 62
MiB = 1 << 20

__all__ = ["calibrate", "fit_alpha_busbw", "choose_routes", "probe_sizes", "enabled", "self_check"]


def enabled(pg) -> bool:
    """``XDDP_COMM_CALIBRATE=1`` on a multi-rank RCCL or peer group that has not been calibrated."""
    return (os.environ.get("XDDP_COMM_CALIBRATE", "0") == "1" and pg.size() > 1
            and pg.backend in ("rccl", "peer") and getattr(pg, "comm_calibration", None) is None)


def probe_sizes(first_bytes: int, cap_bytes: int, tail_bytes: int, total_bytes: int) -> List[int]:
    """The planned bucket sizes plus two latency-bound sizes (64 KiB, 256 KiB), each rounded to
    4 KiB and capped at 256 MiB, ascending."""
    raw = [64 << 10, 256 << 10, first_bytes, tail_bytes, cap_bytes, min(total_bytes, 2 * cap_bytes)]
    out = sorted({max(4096, min(256 * MiB, int(s) // 4096 * 4096)) for s in raw if s and s > 0})
    return out


def fit_alpha_busbw(sizes: Sequence[int], times_s: Sequence[float], world: int) -> Tuple[float, float]:
    """(alpha_us, busbw_GBps) of ``t(S) = alpha + 2 (W-1)/W * S / B`` from measured points.

    alpha = the least-squares intercept, floored at 1 us and capped at the smallest measured time;
    B = the bus bandwidth implied by the largest message after alpha:
    ``B = f * S_max / (t(S_max) - alpha)``. (A plain two-parameter least-squares fit lets the
    small, noisy latency points tilt the slope; the largest message pins B.)"""
    pts = sorted((int(s), float(t)) for s, t in zip(sizes, times_s) if t and t > 0)
    if not pts:
        raise ValueError("no timings to fit")
    f = 2.0 * (max(2, world) - 1) / max(2, world)
    n = len(pts)
    if n >= 2:
        mx = sum(s for s, _ in pts) / n
        my = sum(t for _, t in pts) / n
        sxx = sum((s - mx) ** 2 for s, _ in pts)
        sxy = sum((s - mx) * (t - my) for s, t in pts)
        slope = sxy / sxx if sxx > 0 else 0.0
        alpha = my - slope * mx
    else:
        alpha = pts[0][1]
    alpha = min(max(alpha, 1e-6), pts[0][1])
    s_max, t_max = pts[-1]
    busy = t_max - alpha
    if busy <= 0:
        busy = t_max
    bw = f * s_max / busy
    return round(alpha * 1e6, 3), round(bw / 1e9, 3)


ROUTE_MARGIN = float(os.environ.get("XDDP_ROUTE_MARGIN", "0.1"))


def choose_routes(sizes: Sequence[int], times: Dict[int, Sequence[Optional[float]]]) -> Tuple[List[int], List[int], Dict[int, int]]:
    """Fastest route per probe size -> (bounds, routes, winner_by_size).

    ``times[route][i]`` = seconds at ``sizes[i]`` (None = route unavailable at that size). A peer
    route wins only below (1 - ROUTE_MARGIN) x the base route's time (ties and near-ties go to the
    base route; among peer routes, the faster, then the lower route id). Messages up to
    ``bounds[k]`` bytes take ``routes[k]``; the last bound is open-ended."""
    order = sorted(range(len(sizes)), key=lambda i: sizes[i])
    winner: Dict[int, int] = {}
    # a hand-written peer lane replaces the library path only where it is clearly faster: it must
    # beat the base route's time by ROUTE_MARGIN (measurement noise must not route gradients onto the
    # less-exercised path for a gain of a few percent)
    for i in order:
        base_t = times.get(ROUTE_BASE, [None] * len(sizes))[i]
        best_r, best_t = ROUTE_BASE, (None if base_t is None else base_t * (1.0 - ROUTE_MARGIN))
        for r in sorted(times):
            t = times[r][i]
            if t is None or r == ROUTE_BASE:
                continue
            if best_t is None or t < best_t:
                best_r, best_t = r, t
        winner[int(sizes[i])] = best_r
    ss = [int(sizes[i]) for i in order]
    bounds: List[int] = []
    routes: List[int] = []
    for k, s in enumerate(ss):
        r = winner[s]
        if routes and routes[-1] == r:
            continue
        if routes:  # boundary between the previous segment's last size and this one
            bounds[-1] = int(math.sqrt(ss[k - 1] * s))
        bounds.append(_MAX_BOUND)
        routes.append(r)
    return bounds, routes, winner


# ----------------------------------------------------------------------------------------- device side
def _pattern(n: int, rank: int, k: int, dtype, device) -> torch.Tensor:
    # small integers: every partial sum is exact in fp32 and, below 256, in bf16
    return ((torch.arange(n, device=device) % 13) + 3 * rank + (k % 4)).to(dtype)


def _expected(n: int, world: int, k: int, dtype, device) -> torch.Tensor:
    base = (torch.arange(n, device=device) % 13) * world + 3 * world * (world - 1) // 2 + world * (k % 4)
    return base.to(dtype)


def self_check(pg, iters: int = 8) -> Tuple[bool, str]:
    """Every rank runs the same peer-route all-reduces and checks the exact results; returns
    (this rank's verdict, reason). The caller combines the verdicts across ranks."""
    comm = pg.comm
    routes = list(comm.routes())
    if ROUTE_TWO_SHOT not in routes and ROUTE_ONE_SHOT not in routes:
        return False, "peer lanes not available on this rank"
    rank, world, dev = pg.rank(), pg.size(), pg.device
    corrupt = os.environ.get("XDDP_CALIBRATE_CORRUPT_RANK")  # fault injection (tests)
    corrupt = corrupt is not None and int(corrupt) == rank
    SUM = _redop("SUM")
    one_cap = int(comm.one_shot_capacity())
    bad = []
    try:
        for k in range(iters):
            dt = torch.float32 if k % 2 == 0 else torch.bfloat16
            esz = torch.empty(0, dtype=dt).element_size()
            cases = []
            if ROUTE_TWO_SHOT in routes:
                cases.append((ROUTE_TWO_SHOT, (MiB + (k % 3) * 65536) // esz + 8 * k))
            if ROUTE_ONE_SHOT in routes and one_cap > 0:
                cases.append((ROUTE_ONE_SHOT, min(one_cap, 65536) // esz - 8 * (k % 3)))
            for route, n in cases:
                x = _pattern(n, rank, k, dt, dev)
                comm.allreduce_via(x, SUM, route).wait()
                want = _expected(n, world, k, dt, dev)
                if corrupt and k == 3:
                    want = want + 1
                torch.cuda.synchronize(dev)
                if comm.peer_status() != 0:
                    return False, f"a peer kernel timed out (call {k}, {ROUTE_NAMES[route]})"
                if not torch.equal(x, want):
                    bad.append(f"call {k} {ROUTE_NAMES[route]} {str(dt).replace('torch.', '')} n={n}")
        # a burst without host syncs, the way DDP issues its buckets: both lanes and the base route
        # interleaved, every call on its own tensor and pattern (consecutive uses of a lane's
        # double-buffered slot carry different values), checked only after the whole burst
        burst = []
        for k in range(iters):
            for route, n in ((ROUTE_TWO_SHOT, (2 * MiB) // 4 + 8 * k),
                             (ROUTE_ONE_SHOT, min(one_cap, 65536) // 4 - 4 * k), (ROUTE_BASE, 4096 + 8 * k)):
                if (route != ROUTE_BASE and route not in routes) or n <= 0:
                    continue
                x = _pattern(n, rank, 100 + k, torch.float32, dev)
                burst.append((route, k, x, n, comm.allreduce_via(x, SUM, route)))
        for b in burst:
            b[4].wait()  # (stream order only: no host sync inside the burst)
        torch.cuda.synchronize(dev)
        if comm.peer_status() != 0:
            return False, "a peer kernel timed out (burst)"
        for route, k, x, n, _ in burst:
            if not torch.equal(x, _expected(n, world, 100 + k, torch.float32, dev)):
                bad.append(f"burst call {k} {ROUTE_NAMES[route]} n={n}")
    except RuntimeError as e:
        return False, f"peer route raised: {e}"
    if bad:
        return False, "wrong all-reduce result: " + "; ".join(bad[:3])
    return True, "ok"


def _redop(name):
    from .._native import load

    return getattr(load().RedOp, name)


def _time_route(pg, nbytes: int, route: int, dtype, iters: int) -> float:
    comm = pg.comm
    esz = torch.empty(0, dtype=dtype).element_size()
    buf = torch.ones(max(1, nbytes // esz), dtype=dtype, device=pg.device)
    AVG = _redop("AVG")
    for _ in range(2):
        comm.allreduce_via(buf, AVG, route).wait()
    torch.cuda.synchronize(pg.device)
    pg.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        comm.allreduce_via(buf, AVG, route).wait()
    torch.cuda.synchronize(pg.device)
    return (time.perf_counter() - t0) / iters


def calibrate(pg, sizes: Sequence[int], dtype=torch.bfloat16, iters: int = 5) -> dict:
    """Self-check, time, fit and route (module docstring); returns the report and stores it as
    ``pg.comm_calibration``. No-op report for one rank or a backend without device collectives."""
    from ..parallel import bucket_policy as bp

    one_rank_forced = (pg.size() == 1 and pg.backend == "rccl" and os.environ.get("XDDP_RCCL_FORCE_LAUNCH") == "1"
                       and os.environ.get("XDDP_CALIBRATE_ONE_RANK") == "1")  # (one-GPU test of the RCCL path)
    if (pg.size() <= 1 and not one_rank_forced) or pg.backend not in ("rccl", "peer"):
        rep = {"skipped": f"{pg.backend} backend with {pg.size()} rank(s): nothing to calibrate"}
        pg.comm_calibration = rep
        return rep
    comm = pg.comm
    world = pg.size()
    t_start = time.perf_counter()
    sizes = sorted({int(s) for s in sizes})
    # 1. self-check of the peer lanes, agreed by all ranks
    has_peer = bool(list(comm.routes()))
    # Lanes on probation are self-checked under a short timeout: their failures are not
    # communicator errors and closing them leaves a working base path. RCCL with
    # XDDP_PEER_ALLREDUCE=1/2 arms the lanes at init: they get the same data self-check under their
    # configured (communicator) timeout — a short one would abort the communicator — and a wrong
    # result is fatal on every rank (there is no probation to end, and a lane that maps but reduces
    # wrongly must never carry a gradient). The peer backend has no other path: a failed self-check
    # there is fatal as well (raised on every rank below).
    on_probation = pg.backend == "peer" or comm.info().get("peer_probation", "0") == "1"
    armed = has_peer and not on_probation
    if has_peer and on_probation:
        comm.set_peer_timeout_ms(float(os.environ.get("XDDP_CALIBRATE_TIMEOUT_MS", "5000")))
        ok, reason = self_check(pg)
    elif has_peer:
        ok, reason = self_check(pg)
    else:
        ok, reason = False, "peer lanes not created (XDDP_PEER_ALLREDUCE unset or IPC mapping failed)"
    fail = torch.tensor([0 if ok else 1], dtype=torch.int32, device=pg.device)
    comm.allreduce_via(fail, _redop("MAX"), ROUTE_BASE).wait()
    torch.cuda.synchronize(pg.device)
    all_ok = has_peer and int(fail.item()) == 0
    if has_peer and ok and not all_ok:
        reason = "another rank's self-check failed"
    if armed and not all_ok:
        raise RuntimeError(f"xddp calibrate: the peer lanes armed by XDDP_PEER_ALLREDUCE failed their self-check "
                           f"on rank {pg.rank()} ({reason}); unset XDDP_PEER_ALLREDUCE or use 'auto' (probation)")
    if pg.backend == "peer" and not (ok and all_ok):
        # the verdict all-reduce itself ran on the lane under test; with no fallback path the only
        # safe outcome is to stop every rank before a gradient is all-reduced on it
        raise RuntimeError(f"xddp calibrate: peer backend self-check failed on rank {pg.rank()} "
                           f"({reason}); the peer backend has no fallback path — use the rccl backend")
    if has_peer:
        if all_ok:
            timeout_ms = float(os.environ.get("XDDP_PEER_TIMEOUT_MS", pg.timeout.total_seconds() * 1000))
            if pg.backend == "peer":
                timeout_ms = min(timeout_ms, float(os.environ.get("XDDP_PEER_DEVICE_TIMEOUT_S", "120")) * 1000)
            comm.set_peer_timeout_ms(timeout_ms)
        else:
            comm.finish_peer_probation(False)  # every rank: close the lanes, keep the base path
    # 2. timings on every usable route, MAX-reduced so every rank holds the same matrix
    routes = [ROUTE_BASE]
    if all_ok:
        avail = list(comm.routes())
        if pg.backend == "rccl" and ROUTE_ONE_SHOT in avail:
            routes.append(ROUTE_ONE_SHOT)  # (on the peer backend the base path IS the one-shot lane)
        if ROUTE_TWO_SHOT in avail:
            routes.append(ROUTE_TWO_SHOT)
    one_cap = int(comm.one_shot_capacity()) if all_ok else 0
    mat = torch.full((len(routes), len(sizes)), -1.0, dtype=torch.float64)
    for ri, r in enumerate(routes):
        for si, s in enumerate(sizes):
            if r == ROUTE_ONE_SHOT and s > one_cap:
                continue
            mat[ri, si] = _time_route(pg, s, r, dtype, iters)
    md = mat.to(pg.device).reshape(-1)
    comm.allreduce_via(md, _redop("MAX"), ROUTE_BASE).wait()
    mat = md.cpu().reshape(len(routes), len(sizes))
    times = {r: [None if mat[ri, si] < 0 else float(mat[ri, si]) for si in range(len(sizes))]
             for ri, r in enumerate(routes)}
    # 3. alpha / B of the base path -> the bucket policy
    alpha_us, bw = fit_alpha_busbw(sizes, [t for t in times[ROUTE_BASE]], world)
    bp.set_calibration(alpha_us, bw)
    # 4. route table
    bounds, rts, winner = choose_routes(sizes, times)
    if all_ok:
        comm.set_route_table(bounds, rts)
        comm.finish_peer_probation(True)
    rep = {
        "alpha_us": alpha_us,
        "busbw_GBps": bw,
        "sizes": sizes,
        "timings_ms": {ROUTE_NAMES[r]: [None if t is None else round(t * 1e3, 4) for t in times[r]] for r in routes},
        "route_by_size": {str(s): ROUTE_NAMES[r] for s, r in winner.items()},
        "route_table": ([{"max_bytes": b if b < _MAX_BOUND else None, "route": ROUTE_NAMES[r]}
                         for b, r in zip(bounds, rts)] if all_ok else [{"max_bytes": None, "route": "base"}]),
        "self_check": {"ok": bool(all_ok), "reason": reason if has_peer else reason},
        "backend": pg.backend,
        "seconds": round(time.perf_counter() - t_start, 3),
    }
    pg.comm_calibration = rep
    return rep
