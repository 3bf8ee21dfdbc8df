# usage: bash scripts/gpu_ab_bench.sh TAG "TESTS" "ENV_A" "ENV_B" [rounds] — focused GPU tests, the
# whole GPU suite, then the default C3 bench alternating two environment settings (A/B on one
# box: A B A B ...); lines under gpurun_out/ab_TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_$1
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 400 python -u -m pytest $2 -x -q --timeout 200 --timeout-method thread > $O/pytest_focus.log 2>&1
  rc=$?; tail -2 $O/pytest_focus.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" $O/pytest_focus.log | head -30; exit $rc; }
fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED" $O/pytest_gpu.log | head -30; exit $rc; }
N=${5:-2}
for i in $(seq 1 $N); do
  for E in "$3" "$4"; do
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
    echo "[$E] $(python3 -c "import json; d=json.load(open('$O/bench_$i.json')); print(d['value'], d['step_ms_median'])")"
  done
done
