# usage: bash scripts/gpu_census.sh TAG — rocprofv3 kernel census of the C3 bench (7 steps: 2 warmup
# + 5 timed), per-step milliseconds by kernel into gpurun_out/census_TAG/census.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/census_$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o c -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
tail -1 $O/prof.log | cut -c1-200
python3 - $O <<'EOF'
import csv, sys
o = sys.argv[1]
rows = list(csv.DictReader(open(f"{o}/c_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows) / 7e6
with open(f"{o}/census.txt", "w") as f:
    print(f"kernel time per step (7 steps): {tot:.2f} ms", file=f)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
        print(f"{float(r['TotalDurationNs']) / 7e6:7.3f} ms  {float(r['Calls']) / 7:6.1f}/step  {float(r['AverageNs']) / 1e3:8.1f} us  {r['Name'][:100]}", file=f)
print(open(f"{o}/census.txt").read())
EOF
