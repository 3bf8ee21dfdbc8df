# usage: bash scripts/ab_env.sh VAR  — bench C3 alternating VAR=1 / VAR=0 (2 runs each, same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
V=$1
for i in 1 2; do for v in 1 0; do
  env $V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$V=$v', d['value'], d['ms_per_step'])"
done; done
