"""Debug/safety infrastructure: desync fingerprints, NaN check, flight recorder."""
import os

import pytest
import torch

from _dist_utils import run_ranks


def _w_desync(rank, world):
    from distributeddataparallel_amd import distributed as d

    t = torch.ones(4 + rank)  # ranks disagree on the collective's size
    try:
        d.all_reduce(t)
    except RuntimeError as e:
        assert "desync detected" in str(e), str(e)
    else:
        raise AssertionError("expected a desync error")


def test_desync_detected_with_debug_detail():
    os.environ["XDDP_DEBUG"] = "DETAIL"
    try:
        run_ranks(_w_desync, world=2)
    finally:
        del os.environ["XDDP_DEBUG"]


def _w_nan(rank, world):
    from distributeddataparallel_amd import distributed as d

    t = torch.ones(8)
    d.all_reduce(t)  # clean tensor passes
    if rank == 1:
        t[3] = float("nan")
    assert len(d.get_default_group().flight_records()) >= 1  # records come from the wrapped comm
    try:
        d.all_reduce(t)
    except RuntimeError as e:
        # rank 1 refuses to reduce NaNs; rank 0 then sees its peer drop out of the collective
        assert ("NaN" in str(e)) if rank == 1 else ("NaN" not in str(e)), str(e)
    else:
        assert rank == 0


def test_nan_check():
    os.environ["XDDP_NAN_CHECK"] = "1"
    try:
        run_ranks(_w_nan, world=2)
    finally:
        del os.environ["XDDP_NAN_CHECK"]


def _timeout_worker(rank, world, prefix):
    import json
    import time
    from datetime import timedelta

    import torch

    from distributeddataparallel_amd import distributed as xdist

    os.environ["XDDP_FLIGHT_DUMP_PREFIX"] = prefix
    xdist.init_process_group("cpu", rank=rank, world_size=world, timeout=timedelta(seconds=2))
    t = torch.ones(8)
    xdist.all_reduce(t)  # seq 0 completes on both ranks
    if rank == 0:
        try:
            xdist.all_reduce(t)  # rank 1 never joins: times out
            raise AssertionError("expected a timeout")
        except RuntimeError as e:
            assert "timed out" in str(e) or "closed" in str(e), e
        rec = json.load(open(f"{prefix}{rank}.json"))
        assert rec["rank"] == 0 and rec["backend"] == "cpu"
        states = [e["state"] for e in rec["entries"]]
        assert states[-1] == "failed" and "completed" in states
        assert json.loads(xdist.get_default_group().comm.flight_json())["num_collectives"] >= 2
    else:
        time.sleep(4)
    os._exit(0)  # the mesh is broken; skip the collective teardown


def test_flight_record_dumped_on_collective_timeout(tmp_path):
    from distributeddataparallel_amd.utils.spawn import free_port, spawn

    spawn(_timeout_worker, args=(2, str(tmp_path / "flight_")), nprocs=2,
          env={"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(free_port()), "OMP_NUM_THREADS": "1"})


def _w_desync_in_coalescing(rank, world):
    """Ranks agree on the first collective of a coalescing block and disagree on the second: the
    fingerprint check (run before each collective, grouped or not) reports it on every rank."""
    from distributeddataparallel_amd import distributed as d

    a = torch.ones(8)
    b = torch.ones(16 + 4 * rank)
    with pytest.raises(RuntimeError, match="desync detected"):
        with d.coalescing():
            d.all_reduce(a)
            d.all_reduce(b)
    # the group is closed again and a matching collective still runs
    c = torch.full((4,), float(rank + 1))
    d.all_reduce(c)
    assert torch.equal(c, torch.full((4,), 3.0))


def test_desync_inside_coalescing_block_detected():
    run_ranks(_w_desync_in_coalescing, world=2, env={"XDDP_DEBUG": "DETAIL"})


def _w_helper_fingerprints(rank, world):
    """The device backends' arrangement on CPU ranks: the fingerprints travel over a separate
    helper communicator (own store prefix), the collectives over the wrapped one."""
    from distributeddataparallel_amd import distributed as d
    from distributeddataparallel_amd._native import load

    C = load()
    pg = d.get_default_group()
    helper = C.make_cpu_comm(C.PrefixStore("fp_helper", pg.store), rank, world, 60.0, "127.0.0.1")
    inner = C.make_cpu_comm(C.PrefixStore("fp_inner", pg.store), rank, world, 60.0, "127.0.0.1")
    dbg = C.make_debug_comm(inner, True, False, helper)
    t = torch.full((5,), float(rank))
    dbg.allreduce(t, C.RedOp.SUM, 1.0).wait()
    assert torch.equal(t, torch.full((5,), 1.0))
    n_inner = len(inner.flight_records())
    with pytest.raises(RuntimeError, match="desync detected"):
        dbg.allreduce(torch.ones(3 + rank), C.RedOp.SUM, 1.0).wait()
    assert len(inner.flight_records()) == n_inner  # the mismatched collective never reached the wrapped comm
    dbg.shutdown()


def test_fingerprints_over_helper_communicator():
    run_ranks(_w_helper_fingerprints, world=2)


def _reinit_worker(rank, world, port):
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd._native import load

    C = load()
    store = C.TCPStore("127.0.0.1", port, rank == 0, world, 60.0, False)  # one store for both lives
    for cycle in range(3):
        xdist.init_process_group("cpu", store=store, rank=rank, world_size=world)
        t = torch.full((6,), float(rank + cycle))
        xdist.all_reduce(t)
        assert torch.equal(t, torch.full((6,), float(1 + 2 * cycle))), (cycle, t)
        xdist.barrier()
        xdist.destroy_process_group()


def test_reinit_over_persistent_store():
    """init / destroy three times over ONE store: each generation's keys (communicator bootstrap,
    init barrier) are its own, so no stale address or already-'done' barrier is read."""
    from distributeddataparallel_amd.utils.spawn import free_ports, spawn

    port, master = free_ports(2)  # distinct: two stores bind them
    spawn(_reinit_worker, args=(2, port), nprocs=2,
          env={"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(master), "OMP_NUM_THREADS": "1"})


def _w_coalescing_other_group(rank, world):
    """A blocking collective on another (CPU) group inside an open coalescing() block is not part of
    that block's launch: it completes before returning, and an object collective reads its result."""
    from distributeddataparallel_amd import distributed as d

    other = d.new_group([0, 1])
    a = torch.full((4,), float(rank + 1))
    with d.coalescing():
        d.all_reduce(a)  # deferred: waited when the block closes
        b = torch.full((3,), float(rank + 10))
        assert d.all_reduce(b, group=other) is None
        assert torch.equal(b, torch.full((3,), 21.0)), b  # completed already
        objs = [None, None]
        d.all_gather_object(objs, {"r": rank}, group=other)
        assert objs == [{"r": 0}, {"r": 1}], objs
    assert torch.equal(a, torch.full((4,), 3.0))


def test_coalescing_defers_only_its_own_group():
    run_ranks(_w_coalescing_other_group, world=2)
