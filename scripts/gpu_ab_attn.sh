# usage: bash scripts/gpu_ab_attn.sh TAG LIBTAG... — attention microbench A/B over library variants
# (EA_LIB_NAME=libespnet_amd_<LIBTAG>.so; "cur" = the working tree's) under rocprofv3 kernel
# trace, plus the hipBLASLt kernel names for the step's Linear shapes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
shift
O=gpurun_out/ab_$T
mkdir -p $O
for L in "$@"; do
  if [ "$L" = cur ]; then N=libespnet_amd.so; else N=libespnet_amd_$L.so; fi
  EA_LIB_NAME=$N timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o attn_$L -- python scripts/attn_bwd_bench.py > $O/attn_$L.log 2>&1 || exit 1
  echo "== $L"; grep attn_ $O/attn_$L.log
  python3 -c "
import csv
for r in csv.DictReader(open('$O/attn_${L}_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:80])
"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o blaslt -- python scripts/blaslt_names.py > $O/blaslt.log 2>&1 || exit 1
grep TF/s $O/blaslt.log
python3 -c "
import csv
for r in csv.DictReader(open('$O/blaslt_kernel_stats.csv')):
    print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:160])
"
