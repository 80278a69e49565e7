"""The launch sequence of the last closure in a rocprofv3 kernel trace (development tool).

  python tools/ktrace_seq.py TRACE.csv MARKER [N]

Prints the N launches (default 400) that follow the last occurrence of the kernel whose name contains MARKER
(e.g. the closure's first kernel), one line each: index, duration (us), gap to the previous launch's end (us), grid,
kernel name. Used to attribute the GEMM launches of one closure to their shapes by position.
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    marker, n = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 400
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if not starts:
        sys.exit(f"no kernel matching {marker!r}")
    i0 = starts[-2] if len(starts) > 1 else starts[-1]  # the last complete closure
    prev_end = None
    for k, r in enumerate(rows[i0:i0 + n]):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev_end) / 1e3 if prev_end else 0.0
        prev_end = e
        print(f"{k:4d} {(e - s) / 1e3:8.1f} {gap:6.1f} g{r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r.get('Grid_Size_Z', '1')} "
              f"{r['Kernel_Name'][:90]}")


if __name__ == "__main__":
    main()
