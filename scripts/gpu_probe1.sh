set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/host_probe.py > gpurun_out/host_probe.log 2>&1 && cat gpurun_out/host_probe.log &&
EA_BENCH_TORCH=1 timeout -k 10 300 python scripts/bench_gemm.py > gpurun_out/bench_gemm.log 2>&1; cat gpurun_out/bench_gemm.log
