set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
EA_OVERLAP_WGRAD=0 timeout -k 10 300 python scripts/gemm_census.py c3 > gpurun_out/census.log 2>&1; echo census rc=$?
EA_BENCH_TORCH=1 timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; echo bench_gemm rc=$?
