# usage: bash scripts/gpu_attn_ab.sh   attention GPU tests, then attn fwd/bwd microbench: current vs libespnet_amd_old.so
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_attn.log 2>&1 && tail -2 gpurun_out/pytest_attn.log &&
for i in 1 2; do
  timeout -k 10 120 python scripts/attn_bwd_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/new: /' &&
  EA_LIB_NAME=libespnet_amd_old.so timeout -k 10 120 python scripts/attn_bwd_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/old: /' || exit 1
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "train or optim or adam or checkpoint or model" > gpurun_out/pytest_opt.log 2>&1 && tail -2 gpurun_out/pytest_opt.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log
