# usage: bash scripts/gpu_lds64_ab.sh — C3 bench alternating the 64x128 GEMM ring depth (EA_LDS64_STAGES)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do for v in 2 3 4; do
  EA_LDS64_STAGES=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_s$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_s$v.log').read().strip().splitlines()[-1]);print('EA_LDS64_STAGES=$v', d['value'], d['ms_per_step'], d['loss'])"
done; done
