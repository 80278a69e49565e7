"""Idle time between consecutive kernels of the closure in a rocprofv3 kernel-trace CSV (development tool).

  python tools/ktrace_gaps.py TRACE.csv MARKER [NCLOSURES]

Takes the last NCLOSURES (default 5) complete closures -- each starts at a launch of the kernel whose name contains
MARKER -- and prints per closure the span, the summed kernel time, the idle time between launches, the gap
histogram, and the largest idle contributors by (previous kernel -> next kernel)."""
import csv
import sys
from collections import defaultdict


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marker, nc = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 5
    starts = [i for i, r in enumerate(rows) if marker in r[2]]
    if len(starts) < 2:
        sys.exit(f"fewer than two launches of {marker!r}")
    starts = starts[-(nc + 1):]
    contrib = defaultdict(lambda: [0, 0.0])
    hist = defaultdict(int)
    tot = [0.0, 0.0, 0.0, 0]
    for a, b in zip(starts[:-1], starts[1:]):
        seg = rows[a:b]
        span = (seg[-1][1] - seg[0][0]) / 1e3
        busy = sum(e - s for s, e, _ in seg) / 1e3
        idle = 0.0
        for (s0, e0, n0), (s1, e1, n1) in zip(seg[:-1], seg[1:]):
            gap = max(0, s1 - e0) / 1e3
            idle += gap
            k = "<1" if gap < 1 else "1-2" if gap < 2 else "2-5" if gap < 5 else "5-20" if gap < 20 else ">=20"
            hist[k] += 1
            key = (n0.split("(")[0][:48], n1.split("(")[0][:48])
            contrib[key][0] += 1
            contrib[key][1] += gap
        print(f"closure: {len(seg)} launches, span {span:.1f} us, kernels {busy:.1f} us, idle {idle:.1f} us "
              f"({idle / span * 100:.1f} %)")
        tot[0] += span
        tot[1] += busy
        tot[2] += idle
        tot[3] += len(seg)
    n = len(starts) - 1
    print(f"\nmean over {n}: {tot[3] / n:.0f} launches, span {tot[0] / n:.1f} us, kernels {tot[1] / n:.1f} us, idle "
          f"{tot[2] / n:.1f} us ({tot[2] / tot[0] * 100:.1f} %), {tot[2] / tot[3]:.2f} us per launch")
    print("gaps:", {k: hist[k] // n for k in ("<1", "1-2", "2-5", "5-20", ">=20")}, "per closure")
    print("\nlargest idle contributors (per closure): count, us, previous -> next")
    for key, (c, g) in sorted(contrib.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"  {c // n:4d} {g / n:8.1f}  {key[0]} -> {key[1]}")


if __name__ == "__main__":
    main()
