# usage: bash scripts/gpu_r4a.sh — round-4 first check: the new / changed GPU tests, then the
# default bench line without the CPU baseline (incl. the DP rehearsal leg).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gemm_gpu.py tests/test_inference_gpu.py tests/test_tshadow_gpu.py tests/test_task_gpu.py \
  tests/test_dp_capture_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
