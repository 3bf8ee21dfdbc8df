"""Summarise a rocprofv3 database (rocpd SQLite, `rocprofv3 --kernel-trace --stats -d DIR -o NAME`).

    python scripts/prof_summary.py gpurun_out/prof/r1v3_results.db [--csv profiles/x.csv] [--steps K]
                                   [--grids] [--top 40]

Writes the per-kernel stats table in rocprofv3's kernel_stats.csv format (Name, Calls,
TotalDurationNs, AverageNs, Percentage, MinNs, MaxNs, StdDev) and prints the top kernels;
--steps K divides totals by K to give per-step milliseconds; --grids splits GEMM kernels
by launch grid (one row per GEMM shape class).
"""
from __future__ import annotations

import argparse
import collections
import csv
import math
import sqlite3


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels").fetchall()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--steps", type=float, default=0)
    ap.add_argument("--grids", action="store_true")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--skip-copies", action="store_true", help="drop __amd_rocclr_* (setup H2D copies)")
    a = ap.parse_args()
    rows = load(a.db)
    if a.skip_copies:
        rows = [r for r in rows if not r[0].startswith("__amd_rocclr")]
    by = collections.defaultdict(list)
    for name, dur, gx, gy, gz, wx in rows:
        key = name
        if a.grids and "gemm" in name:
            key = f"{name} grid=({gx // wx},{gy},{gz})"
        by[key].append(dur)
    tot = sum(sum(v) for v in by.values())
    stats = []
    for k, v in by.items():
        s = sum(v)
        mean = s / len(v)
        sd = math.sqrt(sum((x - mean) ** 2 for x in v) / len(v))
        stats.append((k, len(v), s, mean, 100.0 * s / tot, min(v), max(v), sd))
    stats.sort(key=lambda r: -r[2])
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
            for r in stats:
                w.writerow(r)
    div = a.steps or 1.0
    print(f"total kernel time {tot / 1e6:.3f} ms" + (f" = {tot / 1e6 / div:.3f} ms/step" if a.steps else ""))
    for k, n, s, mean, pct, mn, mx, sd in stats[: a.top]:
        print(f"{pct:6.2f}% {n / div:8.1f} calls {s / 1e6 / div:8.3f} ms {mean / 1e3:9.1f} us  {k[:150]}")


if __name__ == "__main__":
    main()
