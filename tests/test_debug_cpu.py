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
