set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo TESTS_OK &&
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && echo BENCH_OK && tail -1 gpurun_out/bench.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r1v3 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 && echo PROF_OK
