# usage: bash scripts/gpu_r4b.sh — round-4 checks: new / changed GPU tests (fault pin, decoder
# fallback, all_invalid, spawn workers, tshadow freeze, bench-shape and C5 parity), then the
# default bench line (DP rehearsal leg included, no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu -rA \
  tests/test_gemm_gpu.py tests/test_inference_gpu.py tests/test_tshadow_gpu.py tests/test_task_gpu.py \
  tests/test_dp_capture_gpu.py tests/test_benched_shapes_gpu.py "tests/test_model_sized_gpu.py::test_sized_bf16_amp_per_tensor[c5_b2]" \
  tests/test_attention_gpu.py -k "not test_gemm_bf16_tiles[ and not test_gemm_layouts" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
