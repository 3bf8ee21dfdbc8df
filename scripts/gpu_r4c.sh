# round-4 check: device beam step tests + decode bench, the spawn diagnostic, then the rest of
# the new tests and the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
  > $O/pytest_gemm.log 2>&1
rc=$?; tail -3 $O/pytest_gemm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_n512.py > $O/gemm_n512.txt 2>&1 || exit 1
cat $O/gemm_n512.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_ctc_th_gpu.py \
  tests/test_inference_gpu.py > $O/pytest_beam.log 2>&1
rc=$?; tail -3 $O/pytest_beam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/decode_bench.py --utts 3 > $O/decode.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/decode_bench.py --utts 3 --host-select >> $O/decode.txt 2>&1 || exit 1
grep "C3 joint" $O/decode.txt
timeout -k 10 500 python -u scripts/diag/spawn_diag.py > $O/spawn.log 2>&1 || { tail -20 $O/spawn.log; exit 1; }
grep -E "^bs" $O/spawn.log
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu -rA \
  tests/test_benched_shapes_gpu.py "tests/test_model_sized_gpu.py::test_sized_bf16_amp_per_tensor[c5_b2]" \
  tests/test_attention_gpu.py tests/test_dp_capture_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
exit $rc
