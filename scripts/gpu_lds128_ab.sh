# usage: bash scripts/gpu_lds128_ab.sh — GEMM tests with the 3-deep 128x128 ring, then C3 bench
# alternating EA_LDS128_STAGES (2 | 3: one-block-per-CU grids on a 3-deep ring)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
EA_LDS128_STAGES=3 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lds128.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_lds128.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in 3 2; do
  EA_LDS128_STAGES=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_t$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_t$v.log').read().strip().splitlines()[-1]);print('EA_LDS128_STAGES=$v', d['value'], d['ms_per_step'], d['loss'])"
done; done
