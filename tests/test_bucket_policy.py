"""xGMI bucket policy: pinned layouts for the north-star models and parity of the Python
planner with the native rebuild (Reducer::assign_rebuilt)."""
import os
import sys

import pytest
import torch

from distributeddataparallel_amd import models
from distributeddataparallel_amd.parallel import bucket_policy as bp

MiB = 1024 * 1024


def _ready_order_sizes(model_fn, dtype=torch.bfloat16):
    with torch.device("meta"):
        m = model_fn()
    ps = [p for p in m.parameters() if p.requires_grad]
    # grad-ready order ~ reverse registration order (the reference's pre-rebuild heuristic)
    return [p.numel() * torch.empty(0, dtype=dtype).element_size() for p in reversed(ps)]


def test_xgmi_plan_numbers():
    p = bp.xgmi_plan(51 * MiB, 8, alpha_us=30, busbw_gbps=350)
    assert p.first_bytes == MiB
    assert p.cap_bytes == 25 * MiB                    # S_eff (~24 MB) < 25 MiB floor
    assert MiB <= p.tail_bytes < 2 * MiB              # a quarter of alpha's worth of bytes (~1.5 MB)
    big = bp.xgmi_plan(16 * 1024 * MiB, 8, alpha_us=30, busbw_gbps=350)
    assert big.cap_bytes == 256 * MiB                 # T/16 clamped to 256 MiB


def test_resnet50_bf16_layout_pinned():
    sizes = _ready_order_sizes(models.resnet50)
    total = sum(sizes)
    plan = bp.xgmi_plan(total, 8, alpha_us=30, busbw_gbps=350)
    lay = bp.assign(sizes, plan)
    by = bp.bucket_bytes(sizes, lay)
    assert sum(by) == total == 51114064
    ref = bp.assign(sizes, bp.reference_plan())
    ref_by = bp.bucket_bytes(sizes, ref)
    # the reference's last bucket holds ~22 MB that cannot overlap backward; the xGMI tail <= ~7 MB
    assert ref_by[-1] > 15 * MiB
    assert by[-1] <= 4 * MiB and by[-1] >= plan.tail_bytes
    assert len(lay) == len(ref) + 1
    assert bp.exposed_tail_us(by, 8) < 0.5 * bp.exposed_tail_us(ref_by, 8)


def test_vit_l16_layout_pinned():
    sizes = _ready_order_sizes(models.vit_l_16)
    total = sum(sizes)
    plan = bp.xgmi_plan(total, 8, alpha_us=30, busbw_gbps=350)
    lay = bp.assign(sizes, plan)
    by = bp.bucket_bytes(sizes, lay)
    assert plan.cap_bytes == pytest.approx(total / 16, rel=0.01)
    assert 14 <= len(lay) <= 20
    assert by[-1] <= 8 * MiB + max(sizes)


def test_llama3_8b_layout_pinned():
    sizes = _ready_order_sizes(lambda: models.llama3_8b(max_seq_len=128))
    total = sum(sizes)
    assert total == 16060522496                  # 8.03 B params in bf16
    plan = bp.xgmi_plan(total, 8, alpha_us=30, busbw_gbps=350)
    lay = bp.assign(sizes, plan)
    ref = bp.assign(sizes, bp.reference_plan())
    assert plan.cap_bytes == 256 * MiB
    assert len(lay) == 50 and len(ref) == 162   # 3x fewer RCCL launches per step
    # The embedding (1 GB) is produced last in backward: no cap can shrink a bucket below one
    # tensor, so the tail is exposed (~5 ms at W=8) unless something hides it. The report must say
    # so, and name the overlapped optimizer when it is on.
    by = bp.bucket_bytes(sizes, lay)
    assert by[-1] == sizes[-1] > plan.tail_bytes
    rep = bp.tail_report(by, plan, 8, overlapped_optimizer=False)
    assert rep["tail_over_cap"] and rep["mitigation"] == "none"
    assert rep["exposed_tail_us_model"] > 4000
    rep = bp.tail_report(by, plan, 8, overlapped_optimizer="tail", tail_chunks=16)
    assert rep["mitigation"].startswith("deferred optimizer") and "16 chunk" in rep["mitigation"]
    assert rep["optimizer_schedule"] == "tail"
    # updates during backward hide nothing under the tail: the report says so
    rep = bp.tail_report(by, plan, 8, overlapped_optimizer="backward")
    assert rep["mitigation"].startswith("none for the tail")


def test_tail_report_small_tail_uses_cap():
    plan = bp.xgmi_plan(100 * MiB, 8, alpha_us=30, busbw_gbps=350)
    rep = bp.tail_report([40 * MiB, 50 * MiB, plan.tail_bytes // 2], plan, 8, overlapped_optimizer=False)
    assert not rep["tail_over_cap"] and rep["mitigation"].startswith("tail cap")
    assert rep["exposed_tail_us_model"] < 60
    assert bp.tail_report([1, 2], plan, 1, False)["exposed_tail_us_model"] == 0.0


def test_native_rebuild_matches_python_planner():
    """Drive the real Reducer rebuild on the fake backend and compare the layout."""
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as dist

    dist.init_process_group("fake", rank=0, world_size=8)
    try:
        torch.manual_seed(0)
        net = torch.nn.Sequential(*[torch.nn.Linear(256, 256) for _ in range(12)])
        ddp = xddp.DDP(net, bucket_policy="xgmi")
        # shrink caps so a small model exercises first/middle/tail buckets
        plan = bp.BucketPlan(100_000, 400_000, 300_000, "xgmi")
        ddp.bucket_plan = plan
        ddp.bucket_bytes_cap, ddp.first_bucket_bytes_cap = plan.cap_bytes, plan.first_bytes
        ddp._build_reducer()
        x = torch.randn(4, 256)
        for _ in range(2):
            ddp(x).sum().backward()
        order = ddp.reducer.grad_ready_order()
        params = list(net.parameters())
        sizes = [params[i].numel() * 4 for i in order]
        want = [[order[i] for i in b] for b in bp.assign(sizes, plan)]
        assert ddp.reducer.bucket_indices() == want
        assert len(want) >= 3
    finally:
        dist.destroy_process_group()


def test_explicit_cap_keeps_reference_semantics():
    plan, explicit = bp.resolve_plan(None, 25, None, 10 ** 9, 8, "rccl")
    assert explicit and plan.policy == "reference" and plan.tail_bytes == 0
    plan, explicit = bp.resolve_plan(None, None, None, 10 ** 9, 8, "cpu")
    assert plan.policy == "reference"
    plan, explicit = bp.resolve_plan(None, None, None, 10 ** 9, 8, "rccl")
    assert plan.policy == "xgmi" and not explicit


def test_rccl_env_defaults_force_nothing(monkeypatch):
    monkeypatch.delenv("NCCL_MAX_NCHANNELS", raising=False)
    monkeypatch.delenv("XDDP_RCCL_MAX_CHANNELS", raising=False)
    assert bp.rccl_env_defaults(1, "rccl") == {}
    assert bp.rccl_env_defaults(8, "rccl") == {}          # no unmeasured channel cap by default
    assert "NCCL_MAX_NCHANNELS" not in os.environ
    monkeypatch.setenv("XDDP_RCCL_MAX_CHANNELS", "48")   # explicit opt-in
    assert bp.rccl_env_defaults(8, "rccl") == {"NCCL_MAX_NCHANNELS": "48"}
    monkeypatch.setenv("NCCL_MAX_NCHANNELS", "64")       # the user's own setting wins
    monkeypatch.setenv("XDDP_RCCL_MAX_CHANNELS", "16")
    assert bp.rccl_env_defaults(8, "rccl") == {}
    assert os.environ["NCCL_MAX_NCHANNELS"] == "64"

