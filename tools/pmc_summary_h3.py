"""Summarise tools/pmc_h3.sh output: per-kernel mean counter values and kernel-trace durations (dev tool)."""
import collections, csv, glob, sys
out = sys.argv[1]
for p in ("p1", "p2"):
    f = glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(p, "no csv"); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(p, k, {c: f"{sum(v)/len(v):.4g}" for c, v in d.items()})
f = glob.glob(f"{out}/kt/**/*kernel_stats.csv", recursive=True)
if f:
    for r in csv.DictReader(open(f[0])):
        print("kt", r["Name"].split("(")[0][-40:], r["Calls"], r["AverageNs"])
