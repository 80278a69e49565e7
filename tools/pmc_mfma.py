#!/usr/bin/env python3
"""MFMA utilisation and held clock of the closure's matrix kernels, one rocprofv3 --pmc pass per
counter over config-3 closures (tools/quick_time.py, T = 2), each pass with --kernel-trace so every dispatch's counter
is divided by its own duration:

  mfma_busy      = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)   (the chip's SIMD-cycles)
  mfma_busy_active_cus = the same over the CUs the launch can occupy (workgroups resident at most, <= 256)
  held_clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration                            (MI355X_MICROARCH.md DVFS item)
  mfma_insts     = SQ_INSTS_MFMA per dispatch; SQ_BUSY_CYCLES per dispatch (SQ busy, summed over the SEs)

  mfma_rate_of_spec = SQ_VALU_MFMA_BUSY_CYCLES / (duration x 2.4 GHz x 1024 SIMDs)   (clock-independent)

GRBM_GUI_ACTIVE / duration reads high on dispatches shorter than ~0.3 ms (MI355X_MICROARCH.md, DVFS give-back): the
closure's GEMMs run 15-70 us, so their held_clock_ghz is an upper bound and mfma_busy a lower one. The held clock under
the fp16x3 main loops is therefore also measured on long dispatches of the same kernels (LONG: tools/gemm_one.py,
65536 x 4608 x 1152 on tiles 48 / 49, ~2 ms each, random operands). This script never touches the GPU itself: every
pass is a child process (rocprofv3 runs the program after `--`).
Usage: python tools/pmc_mfma.py OUTDIR  -> OUTDIR/pmc_mfma.json
"""
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
from collections import defaultdict

COUNTERS = ["SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE", "SQ_INSTS_MFMA", "SQ_BUSY_CYCLES"]
KERNELS = r"k_gemm_h4|k_gemm_h5|k_mlp|k_ablk|k_gemm_bs|k_fixup_ln|k_attn_fwd_mf|k_attn_bwd_mf|k_p2t_mf|k_t2p_mf"
SIMDS, XCDS = 1024, 8


def short(name):
    n = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n).replace("void ", "")


LONG = [("tile48", ["65536", "4608", "1152", "48", "6"]), ("tile49", ["65536", "4608", "1152", "49", "6"])]


def passes(out, root, env, prog, tag, regex):
    """one rocprofv3 --pmc pass per counter (+ --kernel-trace) of `prog`; per (kernel, grid) counter means, durations"""
    per = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> [values]
    dur = defaultdict(list)                          # kernel -> [ns] (all passes)
    durn = defaultdict(list)                         # kernel name alone -> [ns] (fallback if the grid keys differ)
    wgs = {}
    for c in COUNTERS:
        d = os.path.join(out, f"p_{tag}_{c}")
        cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", c, "--kernel-trace", "--kernel-include-regex",
               regex, "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable, "-u"] + prog
        with open(os.path.join(out, f"p_{tag}_{c}.log"), "w") as f:
            rc = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT, env=env, cwd=root).returncode
        print(f"pass {tag} {c}: rc {rc}", flush=True)
        if rc:
            sys.exit(rc)
        cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        for r in csv.DictReader(open(cc[0])):
            k = short(r["Kernel_Name"]) + " grid " + r.get("Grid_Size", "?")
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            try:
                wgs[k] = -(-int(r["Grid_Size"]) // int(r["Workgroup_Size"]))
            except (KeyError, ValueError, ZeroDivisionError):
                pass
        for r in csv.DictReader(open(kt[0])):
            gs = 1
            for ax in ("X", "Y", "Z"):
                gs *= int(r.get("Grid_Size_" + ax, "1") or 1)
            k = short(r["Kernel_Name"]) + " grid " + str(gs)
            dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            durn[short(r["Kernel_Name"])].append(dur[k][-1])
        shutil.rmtree(d, ignore_errors=True)
    return summarise(per, dur, durn, wgs)


def summarise(per, dur, durn, wgs):
    res = {}
    for k, cs in per.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        ns = sorted(dur[k] or durn[k.split(" grid ")[0]])
        if not ns or "GRBM_GUI_ACTIVE" not in m:
            continue
        dmed = ns[len(ns) // 2]
        cyc = m["GRBM_GUI_ACTIVE"] / XCDS
        rec = {"dispatches_per_pass": len(cs.get("GRBM_GUI_ACTIVE", [])), "duration_us_median": dmed / 1e3, "held_clock_ghz": cyc / dmed, "cycles_per_xcd": cyc}
        if k in wgs:
            rec["workgroups"] = wgs[k]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            rec["mfma_busy"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS)
            rec["mfma_rate_of_spec"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (dmed * 2.4 * SIMDS)
            if k in wgs:
                rec["mfma_busy_active_cus"] = rec["mfma_busy"] * 256 / min(256, wgs[k])
        if "SQ_INSTS_MFMA" in m:
            rec["mfma_insts"] = m["SQ_INSTS_MFMA"]
        if "SQ_BUSY_CYCLES" in m:
            rec["sq_busy_cycles"] = m["SQ_BUSY_CYCLES"]
        res[k] = rec
    return res


def main():
    out = os.path.abspath(sys.argv[1])
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, T="2", TMPDIR="/tmp")
    res = passes(out, root, env, [os.path.join(root, "tools", "quick_time.py")], "closure", KERNELS)
    long = {}
    for name, args in LONG:
        r = passes(out, root, dict(env, PRE="1"), [os.path.join(root, "tools", "gemm_one.py")] + args, name,
                   r"k_gemm_h4|k_gemm_h5")
        long[name] = {"shape": "x".join(args[:3]), **max(r.values(), key=lambda x: x["duration_us_median"])}
    with open(os.path.join(out, "pmc_mfma.json"), "w") as f:
        json.dump({"workload": "config-3 closures (tools/quick_time.py, T = 2: decoder + flow stand-in, 69x128x256)",
                   "counters": COUNTERS, "formulas": __doc__.split("\n\n")[1], "kernels": res,
                   "long_gemm": long}, f, indent=1)
    for name, r in long.items():
        print(f"long {name} {r['shape']}: {r['duration_us_median']:.0f} us, clock {r['held_clock_ghz']:.2f} GHz, "
              f"mfma_busy {r.get('mfma_busy', float('nan')):.3f}", flush=True)
    for k, r in sorted(res.items(), key=lambda x: -x[1]["duration_us_median"]):
        print(f"{k[:60]:60s} {r['duration_us_median']:8.1f} us  clock {r['held_clock_ghz']:.2f} GHz  "
              f"mfma_busy {r.get('mfma_busy', float('nan')):.3f}", flush=True)


if __name__ == "__main__":
    main()
