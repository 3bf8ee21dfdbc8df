# usage: bash scripts/gpu_iter.sh <tag> [pytest -k expr]   GPU tests, bench, GEMM microbench, rocprof stats
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r1}; K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG="-k $K"; else KARG=""; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread $KARG > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; [ $rc -ne 0 ] && exit $rc
EA_BENCH_TORCH=0 timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/bench_gemm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o $TAG -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; tail -1 gpurun_out/prof.log; exit $rc
