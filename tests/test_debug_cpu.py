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
