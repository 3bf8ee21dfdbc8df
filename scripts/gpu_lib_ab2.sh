# usage: bash scripts/gpu_lib_ab2.sh — GEMM probe + bench: current build vs libespnet_amd_old.so, alternating
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for L in libespnet_amd.so libespnet_amd_old.so; do
    echo "== $L"
    EA_LIB_NAME=$L timeout -k 10 200 python scripts/blaslt_fwd_probe.py 2>&1 | grep -v amdgpu.ids | sed 's/| hipBLASLt.*//' || exit 1
    EA_LIB_NAME=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>&1 | tail -1 | cut -c80-140 || exit 1
  done
done
