"""Summarise a rocprofv3 kernel_stats.csv into a per-micro-batch table (markdown)."""
import csv
import sys

path = sys.argv[1]
per = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0   # divide totals by this (e.g. micro-batches)
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total GPU kernel time: {tot/1e6:.1f} ms  ({tot/1e6/per:.2f} ms per unit, unit = 1/{per:g})\n")
print("| kernel | calls | total ms | ms/unit | avg us | % |")
print("|---|---|---|---|---|---|")
for r in rows[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    name = r["Name"].replace("|", "/")
    name = name if len(name) < 90 else name[:87] + "..."
    print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs'])/1e6:.1f} | "
          f"{float(r['TotalDurationNs'])/1e6/per:.2f} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.1f} |")
