# usage: bash scripts/gpu_sub.sh TAG — subsampling GPU tests, then bench + rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 300 python -u -m pytest tests/test_subsampling_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_sub.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|assert" gpurun_out/pytest_sub.log | tail -20; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-250; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $1 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; exit $rc
