# CTC prefix kernel v2 + two-level pre-beam: CTC / beam / inference tests, decode bench + trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_ctc_gpu.py \
  tests/test_ctc_th_gpu.py tests/test_inference_gpu.py > $O/pytest_beam.log 2>&1
rc=$?; tail -3 $O/pytest_beam.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/decode_bench.py --utts 3 > $O/decode.txt 2>&1 || exit 1
timeout -k 10 200 python -u scripts/decode_bench.py --utts 3 --single >> $O/decode.txt 2>&1 || exit 1
grep "C3 joint" $O/decode.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o dec -- python scripts/decode_bench.py --utts 2 > $O/dec.log 2>&1 || exit 1
