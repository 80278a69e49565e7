"""Per-(kernel, grid) median durations from a rocprofv3 kernel-trace CSV: python tools/kstats.py TRACE.csv [substr ...]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
keys = sys.argv[2:]
d = defaultdict(list)
for r in rows:
    k = r["Kernel_Name"][:80] + " g" + r["Grid_Size_X"] + "x" + r["Grid_Size_Y"]
    d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    if not keys or any(s in k for s in keys):
        v2 = sorted(v)
        print(f"{len(v):6d} med {v2[len(v) // 2]:9.1f} us  total {sum(v) / 1e3:8.2f} ms  {k}")
