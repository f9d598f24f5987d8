"""bench.py self-launch + self-reporting on the CPU backend (the same code path as the
GPU N>1 run: the parent spawns one fresh child per rank, forwards rank 0's JSON line, and
fails loudly if any rank fails)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra_env=None, args=(), gpus=2):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--device", "cpu",
                           "--model", "mlp", "--steps", "3", "--warmup", "2", *args],
                          capture_output=True, text=True, timeout=240, env=env, cwd="/tmp")


def test_self_launch_reports_one_json_line(tmp_path):
    base = tmp_path / "n1.json"
    base.write_text(json.dumps({"value": 1000.0}) + "\n")
    r = _run(args=("--baseline-json", str(base)))
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["nranks"] == 2 and d["config"]["parallelism"] == "dp2"
    assert d["steps"] == 3 and d["warmup"] == 2 and d["value"] > 0
    assert d["buckets"]["count"] >= 1 and sum(d["buckets"]["bytes"]) > 0
    c = d["comm"]
    # comm is what the collectives themselves took (the CPU backend's worker clock), one sample per
    # bucket all-reduce; overlap can never exceed it
    assert c["collectives_launched"] >= d["buckets"]["count"] and c["timed_iterations"] >= 2
    assert c["avg_backward_comm_ms"] > 0 and 0 <= c["avg_overlap_ms"] <= c["avg_backward_comm_ms"] + 1e-6
    assert c["exposed_comm_ms"] >= 0 and 0 <= c["overlap_pct"] <= 100.0
    assert len(c["per_bucket_comm_ms"]) >= d["buckets"]["count"]
    assert abs(sum(c["per_bucket_comm_ms"]) - c["avg_backward_comm_ms"]) < 0.01 * c["avg_backward_comm_ms"] + 0.01
    assert d["comm_info"]["backend"] == "cpu" and d["comm_info"]["rank_devices"] == [-1, -1]
    assert d["buckets"]["tail"]["tail_bytes"] == d["buckets"]["bytes"][-1]
    assert d["allreduce_busbw"] and all(p["busbw_GBps"] > 0 for p in d["allreduce_busbw"])
    assert d["scaling_efficiency"] == pytest.approx(d["value"] / 2000.0, rel=1e-3)


def test_self_launch_fails_when_a_rank_fails():
    r = _run(extra_env={"XDDP_FAULT_INJECT": "rank=1,step=2,mode=exit,code=7"})
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "failed" in r.stderr


def test_one_rank_reports_no_comm():
    """At N=1 nothing crosses a link: the comm fields are null, not backward compute time."""
    r = _run(gpus=1)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    c = d["comm"]
    assert c["collectives_launched"] == 0
    for k in ("avg_backward_comm_ms", "avg_overlap_ms", "exposed_comm_ms", "overlap_pct", "per_bucket_comm_ms"):
        assert c[k] is None, (k, c)
    assert c["avg_backward_compute_ms"] is not None and c["timed_iterations"] >= 2
    assert "allreduce_busbw" not in d and "warning" not in d
    assert d["buckets"]["tail"]["exposed_tail_us_model"] == 0.0


def test_flop_count_per_sample_matches_survey():
    """bench.py's MFU denominator: model FLOPs of one forward + backward per sample on the meta device
    (~0.22 GFLOP for the reference ResNet-18 at 32x32; ResNet-50 at 224: 3 x ~8.1)."""
    sys.path.insert(0, REPO)
    import bench

    ref = bench.train_flops_per_sample(bench.parse(["--model", "simplecnn", "--image-size", "32",
                                                    "--batch-size", "32"]))
    r50 = bench.train_flops_per_sample(bench.parse(["--model", "resnet50"]))
    assert ref is not None and 0.20e9 < ref < 0.24e9
    assert r50 is not None and 23e9 < r50 < 26e9
