# usage: bash scripts/gpu_attn.sh — attention GPU tests, attn fwd/bwd microbench, model-level GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error|assert" gpurun_out/pytest_attn.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/attn_bwd_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log; exit $rc
