#!/usr/bin/env python
"""Per-kernel VGPR / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage.

usage: python scripts/kernel_resources.py <file.hip> [name-filter]
"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
ninja = open("distributeddataparallel_amd/build/build.ninja").read()
flags = re.search(r"^hipflags = (.*)$", ninja, re.M).group(1).split()
out = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-c", src, "-o", "/tmp/_kr.o",
                      "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: \s*(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    n = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
    n = re.sub(r"xddp::kernels::\(anonymous namespace\)::", "", n)
    n = re.sub(r"\(.*", "", n)
    if filt in n:
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('AGPRs','?'):>3} agpr spill {r.get('VGPRs Spill','?'):>3} "
              f"occ {r.get('Occupancy [waves/SIMD]','?'):>2} scratch {r.get('ScratchSize [bytes/lane]','?'):>4}  {n}")
