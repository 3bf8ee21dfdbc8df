# usage: bash scripts/gpu_f4.sh TAG — inference tests + the C3 decode benchmark (beam 10, joint CTC),
# captured decoder steps (default) and eager incremental steps (EA_DECODE_GRAPH=0)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/f4_$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_inference_gpu.py -x -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" $O/pytest.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/decode_bench.py > $O/decode.log 2>&1 || { tail -20 $O/decode.log; exit 1; }
grep -v amdgpu.ids $O/decode.log
EA_DECODE_GRAPH=0 timeout -k 10 300 python scripts/decode_bench.py > $O/decode_eager.log 2>&1 || { tail -20 $O/decode_eager.log; exit 1; }
grep -v amdgpu.ids $O/decode_eager.log
