# usage: bash scripts/gpu_stream_ab.sh TAG — GPU suite, then the C3 bench under EA_STREAM_WGRAD
# (deferred weight gradients flushed onto the side stream every N blocks; 0 = once at the end)
# and EA_GEMM_BM32 variants, two runs each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sab_$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1 1" "0 1" "2 1" "1 0" "1 1" "0 1"; do
  set -- $cfg
  EA_STREAM_WGRAD=$1 EA_GEMM_BM32=$2 timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > $O/b_$1_$2.json 2> $O/b_$1_$2.err || exit 1
  python3 -c "import json; d=json.load(open('$O/b_$1_$2.json')); print('STREAM=$1 BM32=$2', d['value'], d['ms_per_step'])"
done
