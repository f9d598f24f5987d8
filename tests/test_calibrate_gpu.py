"""Comm calibration on the device (distributed/calibrate.py), two processes sharing cuda:0 over
the ``peer`` backend (RCCL refuses two ranks on one device; the peer backend runs the same peer
kernels and the same calibration steps): the self-check passes and a route table is installed,
and a corrupted self-check on ONE rank makes BOTH ranks drop the two-shot lane (fail-closed),
with the reason reported. Collectives after calibration are still exact."""
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


def test_calibration_corrupted_self_check_falls_back_on_every_rank():
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
