# usage: bash scripts/gpu_lib_ab.sh   full GPU tests, then C3 bench: current lib vs libespnet_amd_old.so (2 runs each)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do for L in libespnet_amd.so libespnet_amd_old.so; do
  EA_LIB_NAME=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_lib.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_lib.log').read().strip().splitlines()[-1]);print('$L', d['value'], d['ms_per_step'])"
done; done
