# usage: bash scripts/gpu_epi.sh TAG — epilogue timelines, GEMM / model / norm tests, two C3 benches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/epi_$1
mkdir -p $O
bash scripts/gpu_timeline.sh epi_$1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py tests/test_norm_gpu.py -m gpu -x -q --timeout 160 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/b_$r.json 2> $O/b_$r.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$r.json')); print('bench', d['value'], d['step_ms_median'])"
done
