"""Grid-size audit of a rocprofv3 kernel trace: per (kernel, grid, workgroup) the calls, total and mean time and the
workgroup count, sorted by total time -- to find launches that leave CUs idle (fewer workgroups than a round).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o k -- python3 bench.py ...
  python3 scripts/grid_audit.py DIR [top]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
path = glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True)[0]
agg = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    g = tuple(int(r.get(f"Grid_Size_{a}", r.get(f"Grid_{a}", 1)) or 1) for a in "XYZ")
    w = tuple(int(r.get(f"Workgroup_Size_{a}", r.get(f"Workgroup_{a}", 1)) or 1) for a in "XYZ")
    wgs = 1
    for gi, wi in zip(g, w):
        wgs *= max(1, gi // max(1, wi))
    key = (r["Kernel_Name"][:70], wgs, w[0] * w[1] * w[2])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = sum(v[1] for v in agg.values())
print(f"total {tot / 1e3:.1f} ms")
print(f"{'kernel':70s} {'WGs':>7s} {'thr':>4s} {'calls':>6s} {'tot ms':>8s} {'avg us':>8s} {'%':>5s}")
for (n, wgs, thr), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{n:70s} {wgs:7d} {thr:4d} {c:6d} {t / 1e3:8.2f} {t / c:8.1f} {100 * t / tot:5.1f}")
