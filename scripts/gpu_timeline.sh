# usage: bash scripts/gpu_timeline.sh TAG — in-kernel timelines (scripts/gemm_timeline.py) of the
# step's one-wave 256x256 GEMMs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tl_$1
mkdir -p $O
for a in "7968 2048 512 1 1 act" "7968 2048 512 1 1 act_nodrop" "7968 2048 512 1 0 dact" "7968 2048 512 1 0 dact_nodrop" "7968 2048 512 1 1 store" "7968 2048 512 1 1 store_drop"; do
  timeout -k 10 120 python scripts/gemm_timeline.py $a >> $O/tl.log 2>&1 || exit 1
done
grep -v amdgpu.ids $O/tl.log
