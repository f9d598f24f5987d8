#!/usr/bin/env python
"""Top kernels of a rocprofv3 kernel_stats CSV: ms per step, calls per step, avg us."""
import csv
import re
import sys

path, steps = sys.argv[1], float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 40
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel ms/step {tot / 1e6 / steps:.3f}")
for r in rows[:n]:
    name = re.sub(r"xddp::kernels::\(anonymous namespace\)::", "", r["Name"])
    name = re.sub(r"\(.*", "", name)[:120]
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms {int(r['Calls']) / steps:6.1f}x {float(r['AverageNs']) / 1e3:9.1f}us"
          f" {100 * float(r['TotalDurationNs']) / tot:5.1f}%  {name}")
