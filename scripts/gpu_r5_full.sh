# usage: bash scripts/gpu_r5_full.sh TAG PART — PART "a": the conv2 forward HBM-traffic passes
# (scripts/gpu_pmc.sh) and the full GPU suite; PART "b": the default bench line (DP rehearsal and
# CPU baseline included) with the fresh traffic file, the rocprofv3 kernel stats of the C3 bench
# and the C5 bench.  Results under gpurun_out/full_TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
O=gpurun_out/full_$T
mkdir -p $O
if [ "$2" = "a" ]; then
  bash scripts/gpu_pmc.sh $T || exit 1
  cat gpurun_out/pmc/pmc_conv2_fwd.json
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
fi
[ -f gpurun_out/pmc/pmc_conv2_fwd.json ] && cp gpurun_out/pmc/pmc_conv2_fwd.json profiles/
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-2500 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o prof -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dp-rehearsal > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
python3 scripts/step_anatomy.py $O/prof_kernel_trace.csv > $O/step_anatomy.txt
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cut -c1-300 $O/bench_c5.json
