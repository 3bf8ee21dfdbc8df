# usage: bash scripts/gpu_pipe4_ab.sh — GEMM tests on the 4-wave kernel, probe shapes + bench: EA_GEMM_PIPE=5 vs 1
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
EA_GEMM_PIPE=5 timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2 || exit 1
for i in 1 2; do
  for P in 5 1; do
    echo "== EA_GEMM_PIPE=$P"
    EA_GEMM_PIPE=$P timeout -k 10 200 python scripts/blaslt_fwd_probe.py 2>&1 | grep -v amdgpu.ids | sed 's/| hipBLASLt.*//' | grep -E "2048x  512|4096" || exit 1
    EA_GEMM_PIPE=$P timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>&1 | tail -1 | cut -c80-140 || exit 1
  done
done
