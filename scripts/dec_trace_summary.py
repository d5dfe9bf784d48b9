"""Per-kernel averages over the last N kernels of a rocprofv3 kernel trace (the decode bench's graph mode runs last)."""
import collections
import csv
import sys

path, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
tail = rows[-n:]
agg = collections.defaultdict(lambda: [0, 0])
for r in tail:
    a = agg[r["Kernel_Name"][:70]]
    a[0] += 1
    a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
span = (int(tail[-1]["End_Timestamp"]) - int(tail[0]["Start_Timestamp"])) / 1e3
print(f"{path}: last {n} kernels, span {span:.0f} us, busy {sum(v[1] for v in agg.values()) / 1e3:.0f} us")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:8]:
    print(f"  {v[0]:5d} x {v[1] / v[0] / 1e3:7.2f} us  {k}")
