# usage: bash scripts/gpu_tile32.sh TAG — the small-M tile A/B at kernel level (rocprofv3 trace of
# scripts/gemm_dec.py) and a kernel census of the C3 step with the 32x128 tile on and off.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t32_$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o dec -- python scripts/gemm_dec.py > $O/gemm_dec.log 2>&1 || exit 1
python scripts/gemm_dec_trace.py $O/dec_kernel_trace.csv
for v in 1 0; do
  EA_GEMM_BM32=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c$v -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$v.log 2>&1 || exit 1
  python3 - $O/c${v}_kernel_stats.csv $v <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
g = [r for r in rows if "gemm_" in r["Name"] or "splitk" in r["Name"]]
tot = sum(float(r["TotalDurationNs"]) for r in g) / 7e6
print(f"BM32={sys.argv[2]}: GEMM kernel time {tot:.3f} ms/step")
for r in sorted(g, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"   {float(r['TotalDurationNs']) / 7e6:6.3f} ms {float(r['Calls']) / 7:6.1f}/step {float(r['AverageNs']) / 1e3:7.1f} us {r['Name'][:70]}")
EOF
done
