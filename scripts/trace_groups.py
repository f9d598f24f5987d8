"""Group a rocprofv3 kernel trace by (kernel, grid): per-iteration time and dispatch count."""
import collections
import csv
import sys

path, iters = sys.argv[1], int(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 50
g = collections.defaultdict(list)
for x in csv.DictReader(open(path)):
    n = x["Kernel_Name"].replace("void ", "", 1).replace("xddp::kernels::(anonymous namespace)::", "").replace("xddp::dev::bf16_t", "bf16")
    n = n.split("(")[0][:80]
    g[(n, x["Grid_Size_X"], x["Grid_Size_Y"], x["Workgroup_Size_X"])].append(int(x["End_Timestamp"]) - int(x["Start_Timestamp"]))
tot = sum(sum(d) for d in g.values())
print(f"total {tot / iters / 1e3:.1f} us/iter")
for (n, gx, gy, wg), d in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
    print(f"{sum(d) / iters / 1e3:8.1f} us/it n/it={len(d) / iters:5.1f} avg {sum(d) / len(d) / 1e3:7.1f} us  grid {gx}x{gy}/{wg}  {n}")
