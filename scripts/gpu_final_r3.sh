# usage: bash scripts/gpu_final_r3.sh TAG — round-end evidence: full GPU suite, conv2-forward PMC
# traffic (gpu_pmc.sh), rocprofv3 kernel stats of the C3 bench, the default bench line (with the
# CPU baseline) and the C5 bench; everything under gpurun_out/final_TAG.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
O=gpurun_out/final_$T
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc.sh $T || exit 1
cp gpurun_out/pmc/pmc_conv2_fwd.json $O/ && grep traffic_bytes $O/pmc_conv2_fwd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o prof -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cut -c1-300 $O/bench_c5.json
