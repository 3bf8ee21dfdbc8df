# usage: bash scripts/gpu_f4slots.sh TAG — inference (f4) run, then EA_PIPE_SLOTS 0 (auto) vs 4 on the C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_f4.sh $1 || exit 1
O=gpurun_out/f4_$1
EA_PIPE_SLOTS=0 timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q -k "grouped or deferred" --timeout 160 --timeout-method thread > $O/pytest_grouped.log 2>&1
rc=$?; tail -1 $O/pytest_grouped.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 4; do
    EA_PIPE_SLOTS=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('SLOTS=$v', d['value'], d['step_ms_median'])"
  done
done
