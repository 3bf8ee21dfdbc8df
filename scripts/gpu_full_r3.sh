# usage: bash scripts/gpu_full_r3.sh TAG — full GPU suite, conv2 / attention kernel census
# (gpu_check_r3.sh microbenchmarks), the conv2-forward HBM traffic passes (gpu_pmc.sh), C3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
O=gpurun_out/full_$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_check_r3.sh $T tests/test_attention_gpu.py || exit 1
bash scripts/gpu_pmc.sh $T || exit 1
cat gpurun_out/pmc/pmc_conv2_fwd.json
