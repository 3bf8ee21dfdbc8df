"""Per-shape GEMM census of a C3 bench run (scripts/gpu_gemm_census.sh): joins the dispatcher's
EA_GEMM_TRACE shape lines with the rocprofv3 kernel trace by (kernel, blocks, grid z).

    python scripts/gemm_trace_census.py gpurun_out/gc_TAG
"""
import collections
import csv
import re
import statistics
import sys

o = sys.argv[1]
shapes = collections.Counter()
for line in open(f"{o}/trace.err"):
    m = re.match(r"\[ea_gemm\] M=(\d+) N=(\d+) K=(\d+) ak=(\d) bk=(\d) nz=(\d+) tile=(\d+)x(\d+) splitk=(\d+) "
                 r"epi=(\d+) geo=(\d+) lds=(\d)", line)
    if m:
        shapes[tuple(int(v) for v in m.groups())] += 1
by_grid = collections.defaultdict(list)
for s, c in shapes.items():
    M, N, K, ak, bk, nz, bm, bn, sk, epi, geo, lds = s
    blocks = -(-M // bm) * -(-N // bn)
    by_grid[(blocks, nz * sk)].append((s, c))

disp = collections.defaultdict(list)
for r in csv.DictReader(open(f"{o}/g_kernel_trace.csv")):
    n = r["Kernel_Name"]
    if "gemm_" not in n and "splitk" not in n:
        continue
    wg = int(r["Workgroup_Size_X"])
    key = (n.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:48],
           int(r["Grid_Size_X"]) // wg, int(r["Grid_Size_Z"]))
    disp[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)

rows = []
for key, ds in disp.items():
    med = statistics.median(ds)
    rows.append((med * len(ds), key, len(ds), med))
rows.sort(reverse=True)
tot = sum(r[0] for r in rows)
print(f"GEMM dispatch time over the run: {tot / 1e3:.2f} ms ({sum(r[2] for r in rows)} dispatches)")
for t, (name, bx, gz), n, med in rows:
    cand = by_grid.get((bx, gz), [])
    flops = [2.0 * s[0] * s[1] * s[2] * s[5] for s, _ in cand]
    tf = f"{flops[0] / med / 1e6:6.0f} TF/s" if len(set(flops)) == 1 and flops else "           "
    desc = "; ".join(f"{s[0]}x{s[1]}x{s[2]} ak{s[3]}bk{s[4]} nz{s[5]} sk{s[8]} epi{s[9]} geo{s[10]} (x{c})"
                     for s, c in cand[:4])
    print(f"{t / 1e3:7.3f} ms {n:5d} x {med:7.1f} us {tf} {name:42s} b={bx:5d} z={gz:3d}  {desc}")
