# usage: bash scripts/gpu_ctchead_ab.sh — model / trainer GPU tests, then C3 bench alternating
# EA_CTC_HEAD_AUX (CTC head GEMM + lse on the auxiliary stream beside the decoder forward)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_head.log 2>&1; rc=$?; tail -1 gpurun_out/pytest_head.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in 1 0; do
  EA_CTC_HEAD_AUX=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_h$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_h$v.log').read().strip().splitlines()[-1]);print('EA_CTC_HEAD_AUX=$v', d['value'], d['ms_per_step'], d['loss'])"
done; done
