"""Per-call kernel time of scripts/gemm_dec.py from its rocprofv3 kernel trace: for each shape,
the auto / 32x128 / 64x128 configs (55 calls each; a call = the GEMM launch + its split-K
combine, if any) and hipBLASLt, median over the last 50 calls.

    python scripts/gemm_dec_trace.py gpurun_out/.../x_kernel_trace.csv
"""
import csv
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
calls = []  # (kind, us)
for r in rows:
    n, d = r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n.startswith("Cijk"):
        calls.append(["blaslt", d, n.split("_MT")[1].split("_")[0]])
    elif "gemm_" in n:
        calls.append(["ours", d, n.split("gemm_")[1].split("(")[0]])
    elif "splitk_reduce" in n and calls and calls[-1][0] == "ours":
        calls[-1][1] += d
        calls[-1][2] += "+splitk"
from gemm_dec import SHAPES  # noqa: E402
i = 0
for M, N, K, bk, kind, _ in SHAPES:
    out = []
    for label in ("auto", "32x128", "64x128", "hipblaslt"):
        grp = calls[i:i + 55]
        i += 55
        ds = sorted(c[1] for c in grp[5:])
        out.append(f"{label}={ds[len(ds) // 2]:5.1f}us[{grp[0][2][:28]}]")
    print(f"{M}x{N}x{K} bk={bk} {kind:5s} " + "  ".join(out))
