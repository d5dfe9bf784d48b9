"""Print a window of a rocprofv3 kernel_trace.csv in launch order (name, duration): e.g. one layer of one
micro-batch, to map library GEMM kernels to the projections that launched them.
  python scripts/prof_sequence.py <kernel_trace.csv> <first_row> <count>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
a, n = int(sys.argv[2]), int(sys.argv[3])
for i, r in enumerate(rows[a:a + n]):
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{a + i:7d} {d:9.1f} us  {r['Kernel_Name'][:110]}")
