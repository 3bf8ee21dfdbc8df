# Round 5 (b): GEMM / DP-capture / B=32 parity tests after the hipBLASLt removal, then the N = 512
# shapes (gemm_k128 K-split wave groups vs the 64x128 tile vs torch's hipBLASLt) and the C3 step
# with gemm_k128 off / on (EA_GEMM_K128=0 / 1), alternated twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py \
  tests/test_dp_ragged_gpu.py tests/test_dp_capture_gpu.py > $O/pytest_a.log 2>&1
rc=$?; tail -3 $O/pytest_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 500 --timeout-method thread \
  "tests/test_benched_shapes_gpu.py::test_c3_b32_fp32_vs_float64" > $O/pytest_b32.log 2>&1
rc=$?; grep "c3 B=32" $O/pytest_b32.log; tail -2 $O/pytest_b32.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u scripts/gemm_n512.py > $O/gemm.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/gemm.txt
for r in 1 2; do
  for k in 0 1; do
    EA_GEMM_K128=$k timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${k}_$r.json 2> $O/b_${k}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${k}_$r.json')); print('k128=$k', d['value'], d['step_ms_median'])" | tee -a $O/bench.txt
  done
done
