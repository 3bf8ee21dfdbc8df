set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_graph.log 2>&1; tail -1 gpurun_out/bench_graph.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --eager > gpurun_out/bench_eager.log 2>&1; tail -1 gpurun_out/bench_eager.log || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1v4 -- python bench.py --steps 5 --warmup 3 --no-cpu-baseline > gpurun_out/prof.log 2>&1; tail -1 gpurun_out/prof.log
