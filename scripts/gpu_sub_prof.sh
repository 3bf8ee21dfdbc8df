# usage: bash scripts/gpu_sub_prof.sh — Conv2dSubsampling fwd+bwd alone (serial wgrad), kernel
# trace with and without the fused conv1-gradient epilogue, summarised per launch grid.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sub
for f in 1 0; do
  EA_FUSE_CONV1_WGRAD=$f EA_OVERLAP_WGRAD=0 timeout -k 10 200 python scripts/sub_bench.py 5 2>&1 | grep -v amdgpu.ids || exit 1
  EA_FUSE_CONV1_WGRAD=$f EA_OVERLAP_WGRAD=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sub -o fuse$f -- python scripts/sub_prof.py 4 > gpurun_out/sub/fuse$f.log 2>&1 || exit 1
  python scripts/trace_grids.py gpurun_out/sub/fuse${f}_kernel_trace.csv 4 || exit 1
done
