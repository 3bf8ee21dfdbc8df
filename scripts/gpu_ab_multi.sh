# usage: bash scripts/gpu_ab_multi.sh TAG REPS "ENV-SET-1" "ENV-SET-2" ... — GPU suite under the
# default env, then the C3 bench under each env set in turn (REPS rounds, interleaved); an env set
# is "VAR=v VAR2=w" (or "-" for the defaults)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abm_$1
mkdir -p $O
reps=$2
shift 2
if [ -z "$AB_SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq $reps); do
  i=0
  for set in "$@"; do
    i=$((i+1))
    e=""; [ "$set" = "-" ] || e="$set"
    env $e timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${i}_$r.json 2> $O/b_${i}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${i}_$r.json')); print('[$set]', d['value'], d['step_ms_median'])"
  done
done
# AB_TRACE="k ...": kernel trace of the bench under each listed env set
for k in $AB_TRACE; do
  set_k="${@:$k:1}"; e=""; [ "$set_k" = "-" ] || e="$set_k"
  env $e timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$k -o trace -- python3 bench.py --steps 10 --warmup 5 --no-cpu-baseline --no-dp-rehearsal > $O/prof_$k.log 2>&1 || exit 1
  find $O/prof_$k -name '*kernel_trace.csv' -exec cp {} $O/kernel_trace_$k.csv \;
  find $O/prof_$k -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_$k.csv \;
  rm -rf $O/prof_$k
done
