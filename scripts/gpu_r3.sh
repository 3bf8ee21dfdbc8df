# usage: bash scripts/gpu_r3.sh <pytest args...>: selected GPU tests, full suite, C3 and C5 bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|Error" gpurun_out/pytest_new.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config c5 --steps 23 > gpurun_out/bench_c5.log 2>&1; rc=$?; tail -1 gpurun_out/bench_c5.log | cut -c1-400; exit $rc
