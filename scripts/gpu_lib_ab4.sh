# usage: bash scripts/gpu_lib_ab4.sh TAG "pytest targets" — the named GPU tests on the current build, then
# the C3 bench alternating libespnet_amd_base.so and the current build (two rounds) and one kernel
# trace of each.  Results under gpurun_out/lab_TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lab_$1
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $2 > $O/pytest.log 2>&1
  rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in 1 2; do
  for L in libespnet_amd_base.so libespnet_amd.so; do
    EA_LIB_NAME=$L timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${L}_$r.json 2> $O/b_${L}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${L}_$r.json')); print('$L', d['value'], d['step_ms_median'])" | tee -a $O/bench.txt
  done
done
for L in libespnet_amd_base.so libespnet_amd.so; do
  EA_LIB_NAME=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o p_$L -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dp-rehearsal > $O/p_$L.json 2> $O/p_$L.err || exit 1
done
