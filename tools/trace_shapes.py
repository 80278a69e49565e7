"""Group a rocprofv3 kernel-trace CSV by (kernel, grid, workgroup) and print calls and mean duration per shape
(dev tool for tools/gpu_trace_shapes.sh)."""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: [0, 0.0])
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r.get("Kernel_Name", "")[:70]
        grid = (r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("Grid_Size_Y", ""), r.get("Grid_Size_Z", ""))
        wg = r.get("Workgroup_Size_X", r.get("Workgroup_Size", ""))
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = (name, grid, wg)
        acc[k][0] += 1
        acc[k][1] += d
rows = sorted(acc.items(), key=lambda kv: -kv[1][1])
tot = sum(v[1] for v in acc.values())
for (name, grid, wg), (n, t) in rows[:80]:
    print(f"{100 * t / tot:6.2f}% {n:6d} {t / n:8.2f}us grid={','.join(grid)} wg={wg} {name}")
