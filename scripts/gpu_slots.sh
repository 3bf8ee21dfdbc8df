# usage: bash scripts/gpu_slots.sh TAG — the GEMM / conv / model tests with the 5-slot ping-pong
# ring (EA_PIPE_SLOTS=5), 4096^3 + step GEMM timings, then the C3 bench A/B 4 vs 5 slots
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/slots_$1
mkdir -p $O
: || EA_PIPE_SLOTS=5 timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_subsampling_gpu.py tests/test_model_gpu.py tests/test_model_sized_gpu.py -m gpu -x -q --timeout 160 --timeout-method thread > $O/pytest5.log 2>&1
rc=$?; tail -1 $O/pytest5.log; [ $rc -eq 0 ] || exit $rc
for v in 4 5; do
  EA_PIPE_SLOTS=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o sub$v -- python scripts/sub_bench.py 5 > $O/sub$v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('$O/sub${v}_kernel_stats.csv')):
    if 'gemm_pipe' in r['Name']: print('slots=$v', r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Name'][40:90])
"
done
for r in 0; do
  for v in 5 4; do
    EA_PIPE_SLOTS=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('SLOTS=$v', d['value'], d['step_ms_median'], d['roofline']['launch_ms'])"
  done
done
timeout -k 10 300 python -u -m pytest tests/test_inference_gpu.py -x -q --timeout 150 --timeout-method thread > $O/pytest_inf.log 2>&1
rc=$?; tail -1 $O/pytest_inf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/decode_bench.py > $O/decode.log 2>&1 || { tail -20 $O/decode.log; exit 1; }
grep -v amdgpu.ids $O/decode.log
EA_DECODE_GRAPH=0 timeout -k 10 300 python scripts/decode_bench.py > $O/decode_eager.log 2>&1 || { tail -20 $O/decode_eager.log; exit 1; }
grep -v amdgpu.ids $O/decode_eager.log
