"""Group a rocprofv3 kernel trace by (kernel, grid): per-iteration time and dispatch count.

usage: python scripts/trace_groups.py TRACE.csv ITERS [TOP] [--steady OPT_KERNEL]

--steady: count only the steady-state steps — the kernels after the first training step's
optimizer kernels (a substring of their name, e.g. sgd_master) up to the last step's — and divide
by the number of steps in that window. Without it every dispatch of the run (model setup, the
initial parameter broadcast, the first step's one-time allocations) is averaged over ITERS.
"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:]]
steady = None
if "--steady" in args:
    k = args.index("--steady")
    steady = args[k + 1]
    del args[k:k + 2]
path, iters = args[0], int(args[1])
top = int(args[2]) if len(args) > 2 else 50
rows = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
if steady:
    pos = [i for i, x in enumerate(rows) if steady in x["Kernel_Name"]]
    groups = [[pos[0]]]
    for p in pos[1:]:
        if p - groups[-1][-1] > 10:
            groups.append([p])
        else:
            groups[-1].append(p)
    if len(groups) < 2:
        raise SystemExit(f"--steady {steady}: fewer than two optimizer steps in the trace")
    rows = rows[groups[0][-1] + 1:groups[-1][-1] + 1]
    iters = len(groups) - 1
g = collections.defaultdict(list)
for x in rows:
    n = x["Kernel_Name"].replace("void ", "", 1).replace("xddp::kernels::(anonymous namespace)::", "").replace("xddp::dev::bf16_t", "bf16")
    n = n.split("(")[0][:80]
    g[(n, x["Grid_Size_X"], x["Grid_Size_Y"], x["Workgroup_Size_X"])].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
tot = sum(sum(d) for d in g.values())
print(f"total {tot / iters / 1e3:.1f} us/iter" + (f" ({iters} steady-state steps)" if steady else ""))
for (n, gx, gy, wg), d in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(d) / iters / 1e3:8.1f} us/it n/it={len(d) / iters:5.1f} avg {sum(d) / len(d) / 1e3:7.1f} us  grid {gx}x{gy}/{wg}  {n}")
