# usage: bash scripts/gpu_ctcbwd_ab.sh — GPU tests, then C3 bench alternating EA_OVERLAP_CTC_BWD
# (CTC head backward forked onto the auxiliary stream beside the decoder backward)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_trainer_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k fork > gpurun_out/pytest_fork.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_fork.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for v in 1 0; do
  EA_OVERLAP_CTC_BWD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_ctc$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_ctc$v.log').read().strip().splitlines()[-1]);print('EA_OVERLAP_CTC_BWD=$v', d['value'], d['ms_per_step'], d['loss'])"
done; done
