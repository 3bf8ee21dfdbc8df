# usage: bash scripts/gpu_sweep.sh — GEMM tests, then the forced-tile sweep (gpurun_out/sweep.log)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/tile_sweep.py 3 > gpurun_out/sweep.log 2>&1; rc=$?; cat gpurun_out/sweep.log | grep -v amdgpu.ids; exit $rc
