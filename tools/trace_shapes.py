"""Per (kernel, grid) mean duration from a rocprofv3 kernel-trace CSV.
  python tools/trace_shapes.py trace.csv [filter-substring] [top]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
g = collections.defaultdict(list)
for r in rows:
    k = r["Kernel_Name"]
    if flt and flt not in k:
        continue
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    g[(k, r["Grid_Size_X"], r["Workgroup_Size_X"])].append(d)
items = sorted(g.items(), key=lambda x: -sum(x[1]))
tot = sum(sum(v) for v in g.values())
for (k, gx, wx), v in items[:top]:
    short = k.replace("_ZN3vlp", "").replace("EEEEvNS_9GemmShapeET3_T4_T5_", "")[:110]
    print(f"{sum(v) / len(v) / 1000:9.1f} us x{len(v):4d} {100 * sum(v) / tot:5.1f}%  wg={int(gx) // int(wx):6d}  {short}")
