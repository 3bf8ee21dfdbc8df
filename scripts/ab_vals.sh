# usage: bash scripts/ab_vals.sh VAR v1 v2 ...   C3 bench for each VAR value (2 rounds, same box)
set -o pipefail
cd $GRAFT_REPO_ROOT
V=$1; shift
for i in 1 2; do for v in "$@"; do
  env $V=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abv.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abv.log').read().strip().splitlines()[-1]);print('$V=$v', d['value'], d['ms_per_step'])"
done; done
