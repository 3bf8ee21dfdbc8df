# usage: bash scripts/gpu_pipe_ab.sh — C3 bench alternating EA_GEMM_PIPE (1: 256x256 ping-pong
# tiles; 3: 128x128 tiles on the ping-pong kernel too)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do for v in 3 1; do
  EA_GEMM_PIPE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_pipe$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_pipe$v.log').read().strip().splitlines()[-1]);print('EA_GEMM_PIPE=$v', d['value'], d['ms_per_step'], d['loss'])"
done; done
