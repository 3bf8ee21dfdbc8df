# usage: bash scripts/gpu_smoke_dp.sh — smoke(), the 2-rank DDP GPU tests, and the N=2 bench path
# rehearsed with two ranks sharing the GPU over gloo (RCCL needs one GPU per rank)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread 2>&1 | tail -1 || exit 1
EA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dp2.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/dp2.log | tail -2 | cut -c1-400; exit $rc
