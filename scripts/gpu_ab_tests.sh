# usage: bash scripts/gpu_ab_tests.sh VAR [pytest -k expr]   GPU tests (subset), then C3 bench A/B of VAR=1/0
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
K=${2:-model}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_env.sh $1
