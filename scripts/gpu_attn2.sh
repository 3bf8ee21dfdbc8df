# usage: bash scripts/gpu_attn2.sh TAG — attention GPU tests, then the C3 attention microbench
# with the original and the pipelined dQ pass (kernel trace), then the whole GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/attn2_$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest_attn.log 2>&1
rc=$?; tail -3 $O/pytest_attn.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_attn.log | head -20; exit $rc; }
for V in 1 0; do
  ATTN_V1=$V timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o v1_$V -- python scripts/attn_bwd_bench.py > $O/bench_v1_$V.log 2>&1 || exit 1
  echo "== ATTN_V1=$V"; grep attn_ $O/bench_v1_$V.log
  python3 -c "
import csv
for r in csv.DictReader(open('$O/v1_${V}_kernel_stats.csv')):
    if 'attn' in r['Name']: print(r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][:70])
"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-200 $O/bench.json
