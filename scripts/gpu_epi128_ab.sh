# usage: bash scripts/gpu_epi128_ab.sh — GPU tests, then C3 bench alternating EA_EPI128 settings
# (one-round 256x256 GEMMs with activation epilogues re-tiled 128x128; gemm.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
EA_EPI128=3 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_trainer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_epi128.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_epi128.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in ${EPI_VALS:-0 1 3 7}; do
  EA_EPI128=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_epi$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_epi$v.log').read().strip().splitlines()[-1]);print('EA_EPI128=$v', d['value'], d['ms_per_step'])"
done; done
