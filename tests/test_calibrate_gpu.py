"""Comm calibration on the device (distributed/calibrate.py), two processes sharing cuda:0 over
the ``peer`` backend (RCCL refuses two ranks on one device; the peer backend runs the same peer
kernels and the same calibration steps): the self-check passes and a route table is installed,
and a corrupted self-check on ONE rank makes BOTH ranks raise (fail-closed: the peer backend's
base path is the lane under test, so there is nothing to fall back to). On the RCCL communicator
a failed self-check closes the lanes on every rank and keeps the ring. Collectives after
calibration are still exact."""
import zlib

import pytest
import torch

from _dist_utils import run_ranks

pytestmark = pytest.mark.gpu
MiB = 1 << 20


def _w_calibrate(rank, world, expect_ok):
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.distributed import calibrate as cal
    from distributeddataparallel_amd.parallel import bucket_policy as bp

    pg = xdist.get_default_group()
    if not expect_ok:
        with pytest.raises(RuntimeError, match="peer backend self-check failed"):
            cal.calibrate(pg, [64 << 10, MiB, 4 * MiB], torch.bfloat16, iters=3)
        bp.clear_calibration()
        return
    try:
        rep = cal.calibrate(pg, [64 << 10, MiB, 4 * MiB], torch.bfloat16, iters=3)
        assert rep["self_check"]["ok"] is expect_ok, rep
        assert rep["alpha_us"] > 0 and rep["busbw_GBps"] > 0
        assert bp.calibration_source() == "measured"
        routes = list(pg.comm.routes())
        if expect_ok:
            assert 3 in routes and "two_shot" in rep["timings_ms"]
            assert len(pg.comm.route_table()[0]) == len(rep["route_table"])
        else:
            assert 3 not in routes and "two_shot" not in rep["timings_ms"], rep
            assert "wrong all-reduce result" in rep["self_check"]["reason"] or \
                "another rank" in rep["self_check"]["reason"], rep
        # every rank holds the same report (MAX-reduced timings -> identical decisions)
        t = torch.tensor([zlib.crc32(str(rep["route_table"]).encode())], dtype=torch.int64, device="cuda")
        m = t.clone()
        pg.allreduce(m, xdist.ReduceOp.MAX).wait()
        torch.cuda.synchronize()
        assert int(m.item()) == int(t.item())
        # the communicator still reduces exactly on whatever route the table picks
        for n in (1000, (3 * MiB) // 4 + 5):
            x = torch.full((n,), float(rank + 1), device="cuda")
            pg.allreduce(x, xdist.ReduceOp.SUM).wait()
            torch.cuda.synchronize()
            assert torch.equal(x.cpu(), torch.full((n,), float(world * (world + 1) // 2)))
    finally:
        bp.clear_calibration()


def test_calibration_peer_backend_self_check_and_routes():
    run_ranks(_w_calibrate, world=2, backend="peer", args=(True,))


def test_calibration_corrupted_self_check_raises_on_every_rank():
    run_ranks(_w_calibrate, world=2, backend="peer", args=(False,), env={"XDDP_CALIBRATE_CORRUPT_RANK": "1"})


def _w_calibrate_rccl_one_rank(rank, world, corrupt):
    """The RCCL communicator's side of the calibration on one GPU: forced RCCL launches at W = 1
    with the peer lanes on probation (XDDP_PEER_ALLREDUCE=auto), allreduce_via on every route, the
    route table, and the probation verdict (kept, or closed after a failed self-check)."""
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.distributed import calibrate as cal
    from distributeddataparallel_amd.parallel import bucket_policy as bp

    pg = xdist.get_default_group()
    assert pg.backend == "rccl" and set(pg.comm.routes()) == {2, 3}
    assert pg.comm_info()["peer_probation"] == "1"
    try:
        rep = cal.calibrate(pg, [64 << 10, MiB, 8 * MiB], torch.bfloat16, iters=3)
        assert rep["self_check"]["ok"] is (not corrupt), rep
        if corrupt:
            assert list(pg.comm.routes()) == [] and rep["route_table"] == [{"max_bytes": None, "route": "base"}]
        else:
            assert pg.comm_info()["peer_probation"] == "0" and set(rep["timings_ms"]) == {"base", "one_shot", "two_shot"}
        for n in (1000, MiB // 2 + 3):  # every route the table picks still reduces exactly (W = 1: identity)
            x = torch.arange(n, device="cuda", dtype=torch.float32)
            pg.allreduce(x, xdist.ReduceOp.SUM).wait()
            torch.cuda.synchronize()
            assert torch.equal(x.cpu(), torch.arange(n, dtype=torch.float32))
    finally:
        bp.clear_calibration()


@pytest.mark.parametrize("corrupt", [False, True])
def test_calibration_rccl_communicator_one_rank(corrupt):
    env = {"XDDP_RCCL_FORCE_LAUNCH": "1", "XDDP_PEER_ALLREDUCE": "auto", "XDDP_CALIBRATE_ONE_RANK": "1"}
    if corrupt:
        env["XDDP_CALIBRATE_CORRUPT_RANK"] = "0"
    run_ranks(_w_calibrate_rccl_one_rank, world=1, backend="rccl", args=(corrupt,), env=env)


def _w_rccl_mixed_routes_ddp(rank, world):
    """DDP buckets on a route table that mixes the peer kernels with RCCL (W = 1, forced RCCL
    launches, the peer lanes of the calibration): small buckets take the two-shot kernel, large
    ones the RCCL ring; gradients stay bitwise those of the plain model (AVG over one rank) for
    several iterations. Then a coalesced burst mixing both routes (at W > 1 the bucket bursts at
    the end of backward are one RCCL group): a peer launch inside the group closes it (the group's
    pending RCCL kernels go out first) and reopens it at the same depth (RcclComm::launch_peer)."""
    import torch.nn.functional as F

    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.distributed import calibrate as cal
    from distributeddataparallel_amd.models import SimpleCNN
    from distributeddataparallel_amd.parallel import bucket_policy as bp

    pg = xdist.get_default_group()
    try:
        rep = cal.calibrate(pg, [64 << 10, MiB], torch.float32, iters=2)
        assert rep["self_check"]["ok"], rep
        pg.comm.set_route_table([3 << 19, 1 << 62], [3, 1])  # <= 1.5 MiB: two-shot, larger: RCCL
        torch.backends.cudnn.deterministic = True
        torch.manual_seed(0)
        model, ref = SimpleCNN().cuda(), SimpleCNN().cuda()
        ddp = xddp.DDP(model, device_ids=[0], bucket_cap_mb=1, first_bucket_cap_mb=0.1)
        for it in range(4):
            ref.load_state_dict(model.state_dict())
            x = torch.randn(16, 3, 32, 32, device="cuda")
            y = torch.randint(0, 10, (16,), device="cuda")
            model.zero_grad(set_to_none=True)
            ref.zero_grad(set_to_none=True)
            F.cross_entropy(ddp(x), y).backward()
            F.cross_entropy(ref(x), y).backward()
            for p, q in zip(model.parameters(), ref.parameters()):
                assert torch.equal(p.grad, q.grad), it
            with torch.no_grad():
                for p in model.parameters():
                    p.sub_(0.01 * p.grad)
        torch.cuda.synchronize()
        sizes = ddp.reducer.bucket_sizes_bytes()  # (after the iteration-0 rebuild)
        assert min(sizes) <= 3 << 19 < max(sizes), sizes  # both routes in use
        ops = [r["op"] for r in pg.flight_records()]
        assert "allreduce_two_shot" in ops and "allreduce" in ops, sorted(set(ops))
        # a coalesced burst mixing both routes (what a bucket burst at the end of backward issues at
        # W > 1): RCCL / two-shot / RCCL / two-shot inside one group, nested one level deeper too
        xs = [torch.arange(n, device="cuda", dtype=torch.float32) for n in (700_000, 1000, 600_000, 70_000)]
        with xdist.coalescing(pg):
            for x in xs[:2]:
                pg.allreduce(x, xdist.ReduceOp.SUM)
            with xdist.coalescing(pg):
                for x in xs[2:]:
                    pg.allreduce(x, xdist.ReduceOp.SUM)
        torch.cuda.synchronize()
        for x in xs:
            assert torch.equal(x, torch.arange(x.numel(), device="cuda", dtype=torch.float32))
        ops = [r["op"] for r in pg.flight_records()][-4:]
        assert ops.count("allreduce_two_shot") == 2, ops
    finally:
        bp.clear_calibration()


def test_rccl_mixed_peer_and_ring_routes_in_ddp_bucket_groups():
    env = {"XDDP_RCCL_FORCE_LAUNCH": "1", "XDDP_PEER_ALLREDUCE": "auto", "XDDP_CALIBRATE_ONE_RANK": "1"}
    run_ranks(_w_rccl_mixed_routes_ddp, world=1, backend="rccl", env=env)
