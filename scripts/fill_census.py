"""Per-kernel-family CU fill of one captured step (rocprofv3 kernel trace): workgroups vs the
256 CUs, and the step's time in launches that cannot fill the chip (grid < 256 workgroups of
>= 256 threads, or < 512 of smaller blocks).  usage: fill_census.py kernel_trace.csv"""
import collections
import csv
import re
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if r["Kind"] == "KERNEL_DISPATCH"]
adam = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
step = rows[adam[-2] + 1: adam[-1] + 1]
t0 = int(step[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in step)
fam = collections.defaultdict(lambda: [0.0, 0, 0])
low = 0.0
for r in step:
    n = re.sub(r"\(anonymous namespace\)::|void ", "", r["Kernel_Name"])[:60]
    wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
    g = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])) // max(1, wg)
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    f = fam[n]
    f[0] += d
    f[1] += 1
    f[2] = g
    if g < (256 if wg >= 256 else 512):
        low += d
print(f"step {(t1 - t0) / 1e3:.1f} us; kernel time in launches with < 256 workgroups: {low:.1f} us")
for n, (d, c, g) in sorted(fam.items(), key=lambda kv: -kv[1][0])[:45]:
    print(f"{d:9.1f} us x {c:3d}  grid {g:6d}  {n}")
