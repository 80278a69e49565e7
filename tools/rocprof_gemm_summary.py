"""Summarise a rocprofv3 --stats kernel_stats.csv for the GEMM classes as bench.py reports them (dev tool).

One bench 'GEMM launch' = one gemm_nt call:
  gemm16 (fp16x3): the A pass (k_rowsplit / k_rowscale / k_gather_scales) + k_gemm_h4 / k_gemm_h5 / k_gemm_h3(m) + their split-K
                   fixups (k_gemm_fixup_sub / _sub16); per call = sum / main-kernel calls
  all:             every GEMM kernel (main + fixups + k_rowscale); per call = sum / main-kernel calls
Usage: rocprof_gemm_summary.py <run_kernel_stats.csv> [out.json]"""
import csv, json, sys

rows = list(csv.DictReader(open(sys.argv[1])))
h3_n = h3_ns = rs_ns = fs_ns = 0
main_n = main_ns = fix_ns = 0
other = {}
for r in rows:
    n, calls, tot = r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])
    if "k_gemm_h3" in n or "k_gemm_h4" in n or "k_gemm_h5" in n:
        h3_n += calls
        h3_ns += tot
        main_n += calls
        main_ns += tot
    elif "k_rowscale" in n or "k_rowsplit" in n or "k_gather_scales" in n:
        rs_ns += tot
        fix_ns += tot
    elif "k_gemm_fixup_sub" in n:
        fs_ns += tot
        fix_ns += tot
    elif "k_gemm_fixup" in n:
        fix_ns += tot
    elif "k_gemm_bs" in n or "k_gemm_nt" in n:
        main_n += calls
        main_ns += tot
    else:
        other[n.split("(")[0][:60]] = {"calls": calls, "total_ms": tot / 1e6, "avg_us": tot / calls / 1e3}
out = {"gemm16_calls": h3_n, "gemm16_h3_ms": h3_ns / 1e6, "gemm16_rowscale_ms": rs_ns / 1e6,
       "gemm16_fixup_ms": fs_ns / 1e6, "gemm16_avg_us_per_call": (h3_ns + rs_ns + fs_ns) / max(h3_n, 1) / 1e3,
       "gemm_calls": main_n, "gemm_main_ms": main_ns / 1e6, "gemm_aux_ms": fix_ns / 1e6,
       "gemm_avg_us_per_call": (main_ns + fix_ns) / max(main_n, 1) / 1e3,
       "top_other": dict(sorted(other.items(), key=lambda kv: -kv[1]["total_ms"])[:8])}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
