# usage: bash scripts/gpu_ab_env.sh TAG VAR "v1 v2 ..." [REPS] — GPU suite, then the C3 bench with
# VAR set to each value in turn (REPS rounds, interleaved)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abenv_$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in $(seq ${4:-2}); do
  for v in $3; do
    env $2=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$2=$v', d['value'], d['step_ms_median'])"
  done
done
