# usage: bash scripts/gpu_attn_prof.sh TAG — attention microbench under rocprofv3 kernel stats, dropout 0.1 and 0
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
for P in 0.1 0.0; do
ATTN_P=$P timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o attn_$1_p$P -- python scripts/attn_bwd_bench.py > gpurun_out/attn_prof.log 2>&1 || exit 1
echo "p=$P"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof/attn_$1_p${P}_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:80])
"
done
