# usage: bash scripts/gpu_new.sh <pytest -k expr or test files...>  run selected GPU tests verbosely, then the whole suite
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?; grep -E "PASS|FAIL|ERROR|worst|flips|Error" gpurun_out/pytest_new.log | tail -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; exit $rc
