# usage: bash scripts/gpu_r4_full.sh TAG — full GPU suite, default bench line (DP rehearsal incl., CPU
# baseline), rocprofv3 kernel stats of the C3 bench, C5 bench; all under gpurun_out/full_TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
O=gpurun_out/full_$T
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-2000 $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o prof -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dp-rehearsal > $O/prof_bench.json 2> $O/prof_bench.err || exit 1
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
cut -c1-300 $O/bench_c5.json
