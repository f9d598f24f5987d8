"""Comm calibration logic (distributed/calibrate.py) on synthetic timings: the alpha / bus-bandwidth
fit, the per-size route table, the probe sizes, and the bucket policy's use of the fit. Pure Python
on identical inputs: every rank computes the same plan and route table (here: two independent
evaluations must agree exactly)."""
import pytest

from distributeddataparallel_amd.distributed import calibrate as cal
from distributeddataparallel_amd.parallel import bucket_policy as bp

MiB = 1 << 20


def _model(alpha_us, bw_gbps, world):
    f = 2.0 * (world - 1) / world
    return lambda s: alpha_us * 1e-6 + f * s / (bw_gbps * 1e9)


def test_fit_recovers_alpha_and_busbw():
    sizes = [64 << 10, 256 << 10, MiB, 25 * MiB, 100 * MiB]
    t = _model(28.0, 410.0, 8)
    a, b = cal.fit_alpha_busbw(sizes, [t(s) for s in sizes], 8)
    assert a == pytest.approx(28.0, rel=1e-6) and b == pytest.approx(410.0, rel=1e-6)
    # noisy small messages must not tilt the bandwidth (pinned by the largest message)
    noisy = [t(s) * (1.3 if s < MiB else 1.0) for s in sizes]
    a2, b2 = cal.fit_alpha_busbw(sizes, noisy, 8)
    assert 1.0 <= a2 <= noisy[0] * 1e6 and b2 == pytest.approx(410.0, rel=0.02)


def test_fit_degenerate_inputs():
    a, b = cal.fit_alpha_busbw([MiB], [50e-6], 2)
    assert a == 50.0 and b > 0
    with pytest.raises(ValueError):
        cal.fit_alpha_busbw([MiB], [None], 2)


def test_choose_routes_segments_and_ties():
    sizes = [64 << 10, 256 << 10, MiB, 25 * MiB, 100 * MiB]
    times = {
        1: [30e-6, 35e-6, 40e-6, 150e-6, 520e-6],      # RCCL ring
        2: [12e-6, 20e-6, 60e-6, None, None],          # one-shot (capacity 1 MiB)
        3: [25e-6, 26e-6, 30e-6, 90e-6, 520e-6],       # two-shot; ties at 100 MiB -> base
    }
    bounds, routes, winner = cal.choose_routes(sizes, times)
    assert winner == {64 << 10: 2, 256 << 10: 2, MiB: 3, 25 * MiB: 3, 100 * MiB: 1}
    assert routes == [2, 3, 1]
    assert bounds[0] == int((256 * 1024 * MiB) ** 0.5) and bounds[1] == int((25 * MiB * 100 * MiB) ** 0.5)
    assert bounds[-1] > 1 << 60
    # deterministic: a second evaluation (another rank) agrees exactly
    assert cal.choose_routes(sizes, times) == (bounds, routes, winner)
    # the base path only (fallback after a failed self-check): one open segment
    b2, r2, _ = cal.choose_routes(sizes, {1: times[1]})
    assert r2 == [1] and len(b2) == 1


def test_choose_routes_margin_keeps_near_ties_on_base():
    """A peer route must beat the base route by ROUTE_MARGIN (10 %): a 5 % gain stays on RCCL."""
    sizes = [MiB, 25 * MiB]
    times = {1: [100e-6, 1000e-6], 3: [95e-6, 850e-6]}
    _, _, winner = cal.choose_routes(sizes, times)
    assert cal.ROUTE_MARGIN == 0.1
    assert winner == {MiB: 1, 25 * MiB: 3}


def test_probe_sizes_cover_plan():
    plan = bp.xgmi_plan(51 * MiB, 8, alpha_us=30, busbw_gbps=350)
    s = cal.probe_sizes(plan.first_bytes, plan.cap_bytes, plan.tail_bytes, 51 * MiB)
    assert s == sorted(s) and s[0] == 64 << 10 and all(x % 4096 == 0 for x in s)
    assert plan.first_bytes in s and plan.cap_bytes in s and max(s) <= 256 * MiB


def test_bucket_policy_uses_measured_fit(monkeypatch):
    monkeypatch.delenv("XDDP_RCCL_ALPHA_US", raising=False)
    monkeypatch.delenv("XDDP_RCCL_BUSBW_GBPS", raising=False)
    try:
        bp.clear_calibration()
        assumed = bp.xgmi_plan(16 << 30, 8)
        assert bp.calibration_source() == "assumed defaults"
        bp.set_calibration(10.0, 900.0)  # a fast fabric: latency-bound size grows with B
        measured = bp.xgmi_plan(16 << 30, 8)
        assert bp.calibration_source() == "measured"
        assert measured.as_dict()["alpha_busbw_source"] == "measured"
        assert measured.tail_bytes != assumed.tail_bytes or measured.cap_bytes != assumed.cap_bytes
        monkeypatch.setenv("XDDP_RCCL_ALPHA_US", "30")  # explicit env beats the measurement
        assert bp.calibration_source() == "env"
    finally:
        bp.clear_calibration()


def test_calibrate_skips_cpu_backend():
    class _PG:
        backend = "cpu"

        def size(self):
            return 2

    pg = _PG()
    assert not cal.enabled(pg)
    rep = cal.calibrate(pg, [MiB])
    assert "skipped" in rep and pg.comm_calibration is rep
