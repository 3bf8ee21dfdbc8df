# usage: bash scripts/gpu_gemm_census.sh TAG — per-shape GEMM census of the C3 step.
#  (1) kernel trace of the captured bench, dispatches joined with the dispatcher's shape lines
#      (EA_GEMM_TRACE) by (kernel, blocks, grid z): scripts/gemm_trace_census.py
#  (2) optional (second arg "events"): one serial eager step, event-timed (scripts/gemm_census.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/gc_$1
mkdir -p $O
EA_GEMM_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o g -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/bench.json 2> $O/trace.err || exit 1
python3 scripts/gemm_trace_census.py $O > $O/census_trace.txt && head -70 $O/census_trace.txt
if [ "$2" = events ]; then
  EA_GEMM_TRACE=1 EA_OVERLAP_WGRAD=0 timeout -k 10 300 python scripts/gemm_census.py c3 > $O/census.txt 2> $O/trace_ev.err || exit 1
  grep -v amdgpu.ids $O/census.txt | head -60
fi
