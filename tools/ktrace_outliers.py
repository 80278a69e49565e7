"""Kernel launches far slower than their kernel's median in a rocprofv3 kernel-trace CSV (the 21 ms
k_gemm_h4 / 31 ms k_gemm_bs maxima of a 44 / 22 us kernel), each with the launches around it, the gaps between them and
its position in the run. Usage: python tools/ktrace_outliers.py TRACE.csv [factor] [min_us]
(default: > 20x the median and > 1000 us)."""
import csv
import statistics
import sys
from collections import defaultdict

path = sys.argv[1]
factor = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 1000.0
rows = []
with open(path) as f:
    for r in csv.DictReader(f):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70],
                     r.get("Grid_Size_X", ""), r.get("Queue_Id", r.get("Stream_Id", ""))))
rows.sort()
t0 = rows[0][0] if rows else 0
med = defaultdict(list)
for s, e, n, g, q in rows:
    med[n].append((e - s) / 1e3)
med = {n: statistics.median(v) for n, v in med.items()}
print(f"{len(rows)} launches, {len(med)} kernels, span {(rows[-1][1] - t0) / 1e9:.2f} s")
hits = [i for i, (s, e, n, g, q) in enumerate(rows) if (e - s) / 1e3 > max(min_us, factor * med[n])]
print(f"{len(hits)} outliers (> {factor:g}x median and > {min_us:g} us)")
for i in hits[:40]:
    s, e, n, g, q = rows[i]
    print(f"\n== {n} grid {g}: {(e - s) / 1e3:.1f} us (median {med[n]:.1f}) at t = {(s - t0) / 1e9:.3f} s, launch {i}")
    for j in range(max(0, i - 4), min(len(rows), i + 3)):
        sj, ej, nj, gj, qj = rows[j]
        gap = (sj - rows[j - 1][1]) / 1e3 if j else 0.0
        mark = ">>" if j == i else "  "
        print(f"{mark} {(sj - t0) / 1e9:9.4f} s  gap {gap:10.1f} us  dur {(ej - sj) / 1e3:9.1f} us  q {qj}  {nj} g{gj}")
