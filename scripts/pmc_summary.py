"""Summarise rocprofv3 --pmc counter_collection CSVs: per kernel, the mean of each counter per
dispatch, the mean dispatch duration, and the derived ratios used in DESIGN.md.

    python scripts/pmc_summary.py gpurun_out/pmc3/r3_attn_p1_counter_collection.csv ...

Derived (per dispatch): wait / issue-stall / active shares of SQ_WAVE_CYCLES; MFMA busy as a
fraction of (GRBM_GUI_ACTIVE / 8 XCDs) x 4 SIMDs x 32 CUs per XCD (SQ_VALU_MFMA_BUSY_CYCLES counts
cycles per SIMD summed over SIMDs); TCC hit rate; FETCH_SIZE doubled (gfx950 tallies 128-B
requests at 64 B, MI355X_MICROARCH.md § HBM) in MB."""
import collections
import csv
import sys


def load(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in paths:
        seen = set()
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            k = k.split("(anonymous namespace)::")[1].rstrip("(") if "anonymous" in k else k
            k = k[:90]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            key = (p, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return acc, dur


def main():
    acc, dur = load(sys.argv[1:])
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        d = sorted(dur[k])[len(dur[k]) // 2]
        print(f"== {k}  (median {d:.1f} us over {len(dur[k])} dispatch-passes)")
        for c in sorted(m):
            print(f"   {c:28s} {m[c]:16.0f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in m:
                    print(f"   {c + ' / WAVE_CYCLES':40s} {m[c] / wc:.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            simd_cycles = m["GRBM_GUI_ACTIVE"] / 8 * 4 * 256
            print(f"   {'MFMA busy / SIMD-cycles (approx)':40s} {m['SQ_VALU_MFMA_BUSY_CYCLES'] / simd_cycles:.3f}")
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   {'LDS bank conflict / LDS active':40s} {m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:.3f}")
        if "TCC_HIT_sum" in m:
            print(f"   {'TCC hit rate':40s} {m['TCC_HIT_sum'] / max(1.0, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
        if "FETCH_SIZE" in m:
            print(f"   {'FETCH_SIZE x2 (MB)':40s} {2 * m['FETCH_SIZE'] / 1024:.1f}")
        if "WRITE_SIZE" in m:
            print(f"   {'WRITE_SIZE (MB)':40s} {m['WRITE_SIZE'] / 1024:.1f}")


if __name__ == "__main__":
    main()
