"""Kernel time of one config-3 closure against its wall time (development tool, run on the GPU box under
rocprofv3 --kernel-trace): eager launches (VAEVAR_GRAPH=0, so every kernel appears in the trace) bracketed by
markers, then the same closure replayed as a graph for the wall time.

  VAEVAR_GRAPH=0 rocprofv3 --kernel-trace --output-format csv -d OUT -o run -- python tools/closure_ktrace.py
  python tools/closure_ktrace.py --analyse OUT/.../run_kernel_trace.csv
"""
import csv
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))


def analyse(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    # closures are separated by idle gaps > 2 ms (the host sleeps between them)
    segs, cur = [], [rows[0]]
    for a, b in zip(rows[:-1], rows[1:]):
        if b[0] - a[1] > 2_000_000:
            segs.append(cur)
            cur = []
        cur.append(b)
    segs.append(cur)
    for s in segs[-3:]:
        span = (s[-1][1] - s[0][0]) / 1e3
        busy = sum(e - b for b, e, _ in s) / 1e3
        print(f"segment: {len(s)} launches, span {span:.1f} us, kernel time {busy:.1f} us")
    # the last single-closure segment: kernel time by kernel, and the launch sequence
    one = [s for s in segs if len(s) < 2000][-1]
    agg = {}
    for b, e, n in one:
        k = n.split("(")[0].replace("void vv::", "").replace("(anonymous namespace)::", "")
        c = agg.setdefault(k, [0, 0.0])
        c[0] += 1
        c[1] += (e - b) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"\none closure: {len(one)} launches, {tot:.1f} us of kernel time")
    for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"  {t:8.1f} us {t / tot * 100:5.1f} % {c:4d} x {t / c:7.1f}  {k[:80]}")
    print("\nsequence:")
    for i, (b, e, n) in enumerate(one):
        print(f"{i:4d} {(e - b) / 1e3:7.1f}  {n.split('(')[0].replace('void vv::', '')[:90]}")


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--analyse":
        analyse(sys.argv[2])
        return
    import torch
    from vaevar import config as C
    from vaevar.engine import DAProblem, LGUnet
    from vaevar.problem import make_problem
    from vaevar.synth import smooth_field

    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow = LGUnet(C.FLOW, 1, 1).load_synthetic()
    prob = DAProblem(dec, make_problem(T=2), flow=flow)
    z = torch.from_numpy(0.3 * smooth_field(5, (1, 32, 128, 256))).cuda()
    g = torch.empty_like(z)
    for _ in range(4):
        prob.closure(z, g)
        torch.cuda.synchronize()
        time.sleep(0.01)
    t0 = time.time()
    n = 10
    for _ in range(n):
        prob.closure(z, g)
    torch.cuda.synchronize()
    print(f"closure wall time (this process's mode): {(time.time() - t0) / n * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
