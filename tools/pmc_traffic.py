"""Per-launch HBM traffic of the GEMM kernels from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

gfx950 corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE/WRITE_SIZE are in KB; FETCH_SIZE reports exactly
half of the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE is exact for 16-B
streaming stores. Usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>
"""
import csv, json, statistics, sys


def per_kernel(path, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        vals.setdefault(r["Dispatch_Id"], [r["Kernel_Name"], 0.0])[1] += float(r["Counter_Value"])
    return vals


f = per_kernel(sys.argv[1], "FETCH_SIZE")
w = per_kernel(sys.argv[2], "WRITE_SIZE")


def summary(keys, what):
    gf = [v for n, v in f.values() if any(k in n for k in keys)]
    gw = [v for n, v in w.values() if any(k in n for k in keys)]
    if not gf or not gw:
        return None
    o = {"kernel": what, "launches_fetch": len(gf), "launches_write": len(gw),
         "fetch_bytes_per_launch_raw": 1024 * statistics.mean(gf),
         "fetch_bytes_per_launch": 2 * 1024 * statistics.mean(gf),
         "write_bytes_per_launch": 1024 * statistics.mean(gw)}
    o["hbm_bytes_per_launch"] = o["fetch_bytes_per_launch"] + o["write_bytes_per_launch"]
    return o


out = {
    # one fp16x3 GEMM = its A pass (k_rowsplit / k_rowscale, or none when the LayerNorm wrote the planes / scales) +
    # the main kernel (k_gemm_h4 tile 48, k_gemm_h3(m)) + fixup: counted per main-kernel launch
    "fp16x3": summary(("k_gemm_h4", "k_gemm_h5", "k_gemm_h3"),
                      "fp16x3 main-kernel launches (k_gemm_h4 + k_gemm_h5 + k_gemm_h3(m))"),
    "k_gemm_h4": summary(("k_gemm_h4",), "k_gemm_h4 (tile 48) launches"),
    "k_gemm_h5": summary(("k_gemm_h5",), "k_gemm_h5 (tile 49) launches"),
    "k_gemm_h3": summary(("k_gemm_h3",), "k_gemm_h3(m) launches"),
    "a_pass": summary(("k_rowsplit", "k_rowscale"), "A split / row-scale passes (k_rowsplit, k_rowscale)"),
    "all": summary(("k_gemm_nt", "k_gemm_bs", "k_gemm_h3", "k_gemm_h4"), "every GEMM main-kernel launch"),
    "note": "FETCH_SIZE doubled (gfx950 wide-load undercount), both in KB -> bytes; means over launches",
}
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out))
