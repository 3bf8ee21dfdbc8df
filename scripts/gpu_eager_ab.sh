# usage: bash scripts/gpu_eager_ab.sh — C3 bench: hipGraph replay (default) vs eager launches
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do for v in graph eager; do
  F=""; [ $v = eager ] && F="--eager"
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $F > gpurun_out/ab_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], d['loss'])"
done; done
