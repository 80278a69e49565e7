"""Aggregate a rocprofv3 kernel trace: GEMM time by (kernel, template args, grid) and other kernels (dev tool)."""
import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: [0, 0.0])
other = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    d = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
    n = r['Kernel_Name']
    if 'gemm' in n:
        wg = int(r['Workgroup_Size_X'])
        key = (n.split('<')[0].split('::')[-1], n.split('<')[1].split('>')[0][:36], int(r['Grid_Size_X']) // wg,
               int(r['Grid_Size_Y']), int(r['Grid_Size_Z']))
        agg[key][0] += 1; agg[key][1] += d
    else:
        other[n.split('(')[0]][0] += 1; other[n.split('(')[0]][1] += d
tot = sum(v[1] for v in agg.values()) + sum(v[1] for v in other.values())
print(f"total kernel time {tot/1e6:.1f} ms")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:28]:
    print("GEMM", k, v[0], f"{v[1]/v[0]/1e3:.1f}us", f"{100*v[1]/tot:.1f}%")
for k, v in sorted(other.items(), key=lambda kv: -kv[1][1])[:12]:
    print(k, v[0], f"{v[1]/v[0]/1e3:.1f}us", f"{100*v[1]/tot:.1f}%")
