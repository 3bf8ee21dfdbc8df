# GEMM tile A/B on the step's Linear shapes + a rocprof kernel census of the C3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python scripts/gemm_n512.py > gpurun_out/gemm_n512.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/gemm_n512.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o r3 -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?; tail -1 gpurun_out/prof.log | cut -c1-200; exit $rc
