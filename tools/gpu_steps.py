#!/usr/bin/env python3
"""One parameterised GPU job for gpurun (replaces the per-experiment tools/gpu_r04*.sh one-offs).

Runs the given steps in order, each under its own time limit, and stops at the first failure (a timeout, an abort or
a fault ends the job: nothing more touches the GPU). Output goes to gpurun_out/<TAG>/<NN>_<kind>.{log,json}.
This driver never touches the GPU itself; every step is a child process (rocprofv3 runs the program after `--`).

  python tools/gpu_steps.py TAG STEP [STEP ...]

steps (one shell word each; arguments after ':' are split on whitespace):
  tests[:EXPR]            pytest -m gpu -x -v (per-test timeout 300 s), -k EXPR if given
  smoke                   __graft_entry__.smoke()
  bench[:ARGS]            python bench.py ARGS > NN_bench.json
  ab:REF.so:N[:ARGS]      N interleaved pairs of bench.py ARGS with VAEVAR_LIB=REF.so ("ref") and the tree's build ("new")
  env:K=V[+K=V]:ARGS      bench.py ARGS with extra environment (e.g. env:VAEVAR_GRID_FUSED=0:--config 5)
  rocprof[:ARGS]          rocprofv3 --kernel-trace --stats of bench.py ARGS; keeps kernel_stats.csv (+ the trace with
                          ARGS containing --trace, as kernel_trace.csv)
  pmc:COUNTER[:ARGS]      rocprofv3 --pmc COUNTER of bench.py ARGS (one counter group per pass); keeps counter_collection.csv
  py:SCRIPT[:ARGS]        python SCRIPT ARGS (tools/quick_time.py, tools/h5_check.py, ...)
  pyenv:K=V[+K=V]:SCRIPT[:ARGS]  the same with extra environment (e.g. VAEVAR_LIB=vae-var_amd/vaevar/ab/x.so)
  ktrace:SCRIPT[:ARGS]    rocprofv3 --kernel-trace of python SCRIPT ARGS, summarised per (kernel, grid) by tools/kstats.py
                          into NN_ktrace.txt (the trace itself is not kept)
  kseq:MARKER:SCRIPT[:ARGS]  the same, listed launch by launch after the second-to-last MARKER kernel
                          (tools/ktrace_seq.py) into NN_kseq.txt
  outliers[:ARGS]         rocprofv3 --kernel-trace of bench.py ARGS; the launches far slower than their kernel's median
                          with their neighbours (tools/ktrace_outliers.py) into NN_outliers.txt (the trace is not kept)
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys
import time

LIMIT = {"tests": 1000, "smoke": 200, "bench": 420, "ab": 900, "env": 420, "rocprof": 420, "pmc": 300, "py": 420,
         "pyenv": 420, "ktrace": 420, "kseq": 420, "outliers": 480}


def run(cmd, out, limit, env=None):
    t0 = time.time()
    with open(out, "w") as f:
        p = subprocess.run(["timeout", "-k", "10", str(limit)] + cmd, stdout=f, stderr=subprocess.STDOUT,
                           env=dict(os.environ, **(env or {})))
    print(f"{os.path.basename(out)}: rc {p.returncode} in {time.time() - t0:.0f}s", flush=True)
    return p.returncode


def main():
    tag, steps = sys.argv[1], sys.argv[2:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.chdir(root)
    od = os.path.join(root, "gpurun_out", tag)
    os.makedirs(od, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    py = sys.executable
    for i, st in enumerate(steps):
        kind, _, rest = st.partition(":")
        base = os.path.join(od, f"{i:02d}_{kind}")
        lim = LIMIT[kind]
        if kind == "tests":
            cmd = [py, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-v", "--timeout", "300",
                   "--timeout-method", "thread"] + (["-k", rest] if rest else [])
            rc = run(cmd, base + ".log", lim)
        elif kind == "smoke":
            rc = run([py, "-c", "import __graft_entry__ as g; g.smoke()"], base + ".log", lim)
        elif kind == "bench":
            rc = run([py, "bench.py"] + rest.split(), base + ".json", lim)
        elif kind == "env":
            kv, _, args = rest.partition(":")
            env = dict(x.split("=", 1) for x in kv.split("+") if x)
            rc = run([py, "bench.py"] + args.split(), base + ".json", lim, env)
        elif kind == "ab":
            ref, _, r2 = rest.partition(":")
            n, _, args = r2.partition(":")
            rc = 0
            for k in range(int(n)):
                for arm, env in (("ref", {"VAEVAR_LIB": os.path.abspath(ref)}), ("new", None)):
                    rc = run([py, "bench.py"] + args.split(), f"{base}_{arm}{k}.json", lim // (2 * int(n)), env)
                    if rc:
                        break
                if rc:
                    break
        elif kind in ("rocprof", "pmc"):
            d = base + "_rp"
            if kind == "rocprof":
                prof = ["--kernel-trace", "--stats"]
                args = rest
            else:
                counter, _, args = rest.partition(":")
                prof = ["--pmc"] + counter.split(",")
            cmd = ["rocprofv3"] + prof + ["--output-format", "csv", "-d", d, "-o", "run", "--", py, "bench.py"]
            cmd += [a for a in args.split() if a != "--trace"]
            rc = run(cmd, base + ".log", lim)
            for pat, name in (("*kernel_stats.csv", "kernel_stats.csv"), ("*counter_collection.csv", "counter_collection.csv")) + \
                    ((("*kernel_trace.csv", "kernel_trace.csv"),) if "--trace" in args.split() else ()):
                for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
                    shutil.copy(f, f"{base}_{name}")
            shutil.rmtree(d, ignore_errors=True)
        elif kind in ("ktrace", "kseq"):
            marker = None
            if kind == "kseq":
                marker, _, rest = rest.partition(":")
            script, _, args = rest.partition(":")
            d = base + "_rp"
            cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--", py, "-u",
                   script] + args.split()
            rc = run(cmd, base + ".log", lim)
            if rc == 0:
                tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
                tool = [os.path.join(root, "tools", "kstats.py"), tr[0]] if tr and not marker else \
                    [os.path.join(root, "tools", "ktrace_seq.py"), tr[0], marker, "700"] if tr else None
                rc = run([py] + tool, base + ".txt", 120) if tool else 1
            shutil.rmtree(d, ignore_errors=True)
        elif kind == "outliers":
            d = base + "_rp"
            cmd = ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "run", "--", py, "bench.py"]
            rc = run(cmd + rest.split(), base + ".log", lim)
            if rc == 0:
                tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
                rc = run([py, os.path.join(root, "tools", "ktrace_outliers.py"), tr[0]], base + ".txt", 300) if tr else 1
            shutil.rmtree(d, ignore_errors=True)
        elif kind == "py":
            script, _, args = rest.partition(":")
            rc = run([py, "-u", script] + args.split(), base + ".log", lim)
        elif kind == "pyenv":
            kv, _, r2 = rest.partition(":")
            script, _, args = r2.partition(":")
            env = dict(x.split("=", 1) for x in kv.split("+") if x)
            rc = run([py, "-u", script] + args.split(), base + ".log", lim, env)
        else:
            sys.exit(f"unknown step {st!r}")
        if rc:
            print(f"step {st!r} failed (rc {rc}); stopping", flush=True)
            sys.exit(rc)


if __name__ == "__main__":
    main()
