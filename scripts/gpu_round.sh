# usage: bash scripts/gpu_round.sh <tag>   GPU tests, bench, GEMM census, rocprof kernel stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/gemm_census.py > gpurun_out/census.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/census.log | head -60; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o $TAG -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; tail -1 gpurun_out/prof.log; exit $rc
