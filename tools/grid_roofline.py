"""Config 5's grid-kernel HBM roofline record (profiles/rNN/grid_roofline.json, read by bench.py's config5
sub-record) from a rocprofv3 --kernel-trace --stats run and two --pmc passes (FETCH_SIZE, WRITE_SIZE) of
`bench.py --config 5 ...` (dev tool).

  grid_roofline.py <kernel_stats.csv> <fetch counter_collection.csv> <write counter_collection.csv> <out.json>

Algorithmic bytes (SURVEY §8 d): per evaluation at 721x1440, T = 2, the 7 dense fp32 state fields once each
(xb + yo, H, R per slot) = 2.006 GB; k_misfit_grid reads them in two launches (slot 0: 4 fields, slot 1: 3).
FETCH_SIZE is doubled (gfx950: wide 16-B/lane reads count half, MI355X_MICROARCH.md §HBM), both counters in KB.
"""
import csv
import json
import statistics
import sys

stats, fpath, wpath, out = sys.argv[1:5]
rows = {r["Name"]: r for r in csv.DictReader(open(stats))}


def stat(sub):
    """calls / mean / total over every template instance whose name contains sub"""
    rs = [r for n, r in rows.items() if sub in n]
    if not rs:
        return None
    calls = sum(int(r["Calls"]) for r in rs)
    tot = sum(float(r["TotalDurationNs"]) for r in rs)
    return {"calls": calls, "avg_us": tot / calls / 1e3, "total_ms": tot / 1e6,
            "instances": {n: {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
                          for n, r in rows.items() if sub in n}}


def per_dispatch(path, counter, sub):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and sub in r["Kernel_Name"]:
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


g = stat("k_misfit_grid")
nb = stat("k_misfit_net_bwd")
f = per_dispatch(fpath, "FETCH_SIZE", "k_misfit_grid")
w = per_dispatch(wpath, "WRITE_SIZE", "k_misfit_grid")
alg_launch = 2.006e9 / 2  # bytes per k_misfit_grid launch, averaged over the two slots (4 and 3 fields)
fetch = 2 * 1024 * statistics.mean(f) if f else None
write = 1024 * statistics.mean(w) if w else None
evals = g["calls"] / 2 if g else None  # two k_misfit_grid launches (one per slot) per evaluation
grid_ms = (g["total_ms"] + (nb["total_ms"] if nb else 0.0)) / evals if g else None
misfit_ms = g["total_ms"] / evals if g else None
rec = {
    "source": "rocprofv3 --kernel-trace --stats and --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py --config 5",
    "rocprof": {"k_misfit_grid": g, "k_misfit_net_bwd": nb, "evaluations": evals,
                "grid_ms_per_eval": grid_ms, "k_misfit_grid_ms_per_eval": misfit_ms,
                "achieved_GBs": 2.006e9 / (misfit_ms * 1e-3) / 1e9 if g else None,
                "frac_of_8TBs": 2.006e9 / (misfit_ms * 1e-3) / 8e12 if g else None},
    "algorithmic_bytes_per_launch": alg_launch,
    "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
    "traffic_bytes_per_launch": (fetch or 0) + (write or 0) if f and w else None,
    "traffic_bytes_per_eval": 2 * ((fetch or 0) + (write or 0)) if f and w else None,
    "launches_counted": [len(f), len(w)],
    "note": "achieved = SURVEY 8d's 2.006 GB per evaluation / the k_misfit_grid time per evaluation (both slots); "
            "FETCH_SIZE doubled (gfx950 wide-read undercount), KB -> bytes; means over k_misfit_grid dispatches",
}
json.dump(rec, open(out, "w"), indent=1)
print(json.dumps(rec))
