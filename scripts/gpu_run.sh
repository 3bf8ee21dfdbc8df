# usage: bash scripts/gpu_run.sh "<pytest -k expr or ALL or NONE>" "<bench args or NONE>" [prof]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="$1"; BARGS="$2"; PROF="$3"
if [ "$K" != "NONE" ]; then
  if [ "$K" = "ALL" ]; then timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
  else timeout -k 10 900 python -m pytest tests -m gpu -x -q -k "$K" > gpurun_out/pytest_gpu.log 2>&1; fi
  rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "$BARGS" != "NONE" ]; then
  timeout -k 10 400 python bench.py $BARGS > gpurun_out/bench.log 2>&1; rc=$?; tail -3 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o $PROF -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; tail -2 gpurun_out/prof.log; exit $rc
fi
