# gemm_k128 correctness + N=512 tile A/B, then the beam tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gemm_gpu.py -k k128 \
  > $O/pytest_k128.log 2>&1
rc=$?; tail -3 $O/pytest_k128.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_n512.py > $O/gemm_n512.txt 2>&1 || exit 1
grep -v amdgpu.ids $O/gemm_n512.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_ctc_th_gpu.py \
  > $O/pytest_beam.log 2>&1
rc=$?; tail -3 $O/pytest_beam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/decode_bench.py --utts 3 > $O/decode.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/decode_bench.py --utts 3 --host-select >> $O/decode.txt 2>&1 || exit 1
grep "C3 joint" $O/decode.txt
