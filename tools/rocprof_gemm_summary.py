"""Summarise a rocprofv3 --stats kernel_stats.csv for the GEMM class as bench.py reports it (dev tool):
one bench 'GEMM launch' = one gemm_nt call = the main kernel (k_gemm_bs / k_gemm_nt) plus, for split-K tails,
its k_gemm_fixup; the average per call is (main + fixup time) / main-kernel calls.
Usage: rocprof_gemm_summary.py <run_kernel_stats.csv> [out.json]"""
import csv, json, sys

rows = list(csv.DictReader(open(sys.argv[1])))
main_n = main_ns = fix_ns = 0
other = {}
for r in rows:
    n, calls, tot = r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])
    if "k_gemm_fixup" in n:
        fix_ns += tot
    elif "k_gemm_bs" in n or "k_gemm_nt" in n:
        main_n += calls
        main_ns += tot
    else:
        other[n.split("(")[0][:60]] = {"calls": calls, "total_ms": tot / 1e6, "avg_us": tot / calls / 1e3}
out = {"gemm_calls": main_n, "gemm_main_ms": main_ns / 1e6, "gemm_fixup_ms": fix_ns / 1e6,
       "gemm_avg_us_per_call": (main_ns + fix_ns) / max(main_n, 1) / 1e3,
       "top_other": dict(sorted(other.items(), key=lambda kv: -kv[1]["total_ms"])[:8])}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
