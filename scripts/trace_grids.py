"""Per-(kernel, grid) totals of a rocprofv3 kernel trace CSV, divided by an iteration count.

    python scripts/trace_grids.py trace.csv [iters] [top]
"""
import collections
import csv
import sys

path = sys.argv[1]
iters = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
agg = collections.defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(path)):
    key = (r["Kernel_Name"][:90], int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])), r["Grid_Size_Z"])
    agg[key][0] += 1
    agg[key][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for (name, blocks, gz), (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
    print(f"{us / iters:9.1f} us/iter {n / iters:5.1f} calls {us / n:8.1f} us/call  blocks {blocks}x{gz}  {name}")
