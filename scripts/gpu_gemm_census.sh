# usage: bash scripts/gpu_gemm_census.sh TAG — per-shape GEMM census of one serial C3 step
# (scripts/gemm_census.py, event-timed) with the dispatcher's tile choices (EA_GEMM_TRACE).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gc_$1
mkdir -p $O
EA_GEMM_TRACE=1 EA_OVERLAP_WGRAD=0 timeout -k 10 300 python scripts/gemm_census.py c3 > $O/census.txt 2> $O/trace.err || exit 1
grep -v amdgpu.ids $O/census.txt | head -60
sort $O/trace.err | uniq -c | sort -rn | head -70 > $O/tiles.txt
