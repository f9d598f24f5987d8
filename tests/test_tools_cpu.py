"""The profile post-processing tools behind the committed r3 profiles, on synthetic rocprofv3
CSVs: scripts/overlap_trace.py (overlapped optimizer vs the tail all-reduce) and
scripts/pmc_summary.py (per-op roofline from marker-delimited dispatches)."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TRACE_COLS = ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]


def _write_trace(d, rows):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=TRACE_COLS)
        w.writeheader()
        for i, (name, s, e) in enumerate(rows):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": name, "Start_Timestamp": s, "End_Timestamp": e})


def _run(*args):
    r = subprocess.run([sys.executable, *args], capture_output=True, text=True, timeout=60, cwd=REPO)
    assert r.returncode == 0, r.stderr
    return r.stdout


def test_overlap_trace_counts_updates_around_the_tail(tmp_path):
    ms = 1_000_000
    rows = []
    for it in range(2):  # two iterations, 100 ms apart
        t0 = it * 100 * ms
        rows += [("oneRankReduce<float>", t0 + 1 * ms, t0 + 2 * ms),    # bucket 0
                 ("adam_kernel<bf16>", t0 + 2 * ms, t0 + 3 * ms),       # its update, before the tail
                 ("oneRankReduce<float>", t0 + 4 * ms, t0 + 8 * ms),    # tail bucket
                 ("adam_kernel<bf16>", t0 + 5 * ms, t0 + 6 * ms),       # an update under the tail
                 ("adam_kernel<bf16>", t0 + 8 * ms, t0 + 10 * ms)]      # the tail's own update
    _write_trace(str(tmp_path / "t"), rows)
    out = _run("scripts/overlap_trace.py", str(tmp_path / "t"))
    lines = [l.split() for l in out.splitlines() if l.strip() and l.split()[0].isdigit()]
    assert len(lines) == 2
    for f in lines:  # iter, allreduces, tail ms, during, ms under tail, before, after, last-after ms
        assert f[1] == "2" and float(f[2]) == 4.0 and f[3] == "1" and float(f[4]) == 1.0
        assert f[5] == "1" and f[6] == "1" and float(f[7]) == 2.0


def test_pmc_summary_segments_by_marker(tmp_path):
    us = 1000
    mark = "void at::native::vectorized_elementwise_kernel<short add>"
    rows = [(mark, 0, 1), ("gemm_nt_kernel<256, 0>", 10 * us, 110 * us), ("gemm_nt_kernel<256, 0>", 120 * us, 220 * us),
            (mark, 230 * us, 231 * us), (mark, 300 * us, 301 * us), ("Cijk_MT256x256", 310 * us, 360 * us),
            (mark, 400 * us, 401 * us)]
    _write_trace(str(tmp_path / "t"), rows)
    plan = [{"label": "own", "pattern": "gemm_nt_kernel", "calls": 2, "flops": 2.5e11, "bytes": 1e8},
            {"label": "blas", "pattern": "Cijk", "calls": 1, "flops": 2.5e11, "bytes": 1e8}]
    with open(tmp_path / "plan.json", "w") as f:
        json.dump(plan, f)
    out = _run("scripts/pmc_summary.py", "--plan", str(tmp_path / "plan.json"), "--trace", str(tmp_path / "t"))
    rows = {l.split()[0]: l.split() for l in out.splitlines() if l.startswith(("own", "blas"))}
    assert float(rows["own"][1]) == 100.0 and float(rows["blas"][1]) == 50.0  # us per call
    assert float(rows["own"][2]) == 2500.0 and float(rows["blas"][2]) == 5000.0  # TF/s
