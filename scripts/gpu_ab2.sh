# usage: bash scripts/gpu_ab2.sh TAG VAR "v1 v2" "pytest targets" — the named GPU tests, then the C3
# bench with VAR set to each value in turn (two rounds, interleaved), then a kernel trace of
# the default build.  Results under gpurun_out/ab_TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab_$1
mkdir -p $O
if [ -n "$4" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread $4 > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for v in $3; do
    env $2=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('$2=$v', d['value'], d['step_ms_median'])" | tee -a $O/bench.txt
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o prof -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dp-rehearsal > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/step_anatomy.py $O/prof_kernel_trace.csv > $O/anatomy.txt
head -40 $O/anatomy.txt
