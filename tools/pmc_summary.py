"""Per-kernel mean of each PMC counter over the dispatches whose name matches a filter (dev tool).
Usage: pmc_summary.py <filter> <counter_collection.csv>..."""
import collections, csv, sys

flt = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for path in sys.argv[2:]:
    per = collections.defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        if flt not in r["Kernel_Name"]:
            continue
        k = (r["Dispatch_Id"], r["Counter_Name"])
        per[k] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0][-60:]
    for (d, c), v in per.items():
        agg[names[d]][c].append(v)
for kname, cs in agg.items():
    print(kname)
    for c, vs in sorted(cs.items()):
        print(f"   {c:32s} {sum(vs) / len(vs):16.1f}  (n={len(vs)})")
