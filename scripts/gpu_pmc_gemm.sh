# usage: bash scripts/gpu_pmc_gemm.sh M N K ak bk   — SQ counter passes for one GEMM shape, lds vs pipe kernel
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcg
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
for pipe in 0 1; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    EA_TILE=256 EA_PIPE=$pipe timeout -s KILL 90 rocprofv3 --pmc $P --kernel-include-regex 'gemm_' --output-format csv -d gpurun_out/pmcg -o p${pipe}_pass$i -- python scripts/gemm_one.py "$@" 10 > gpurun_out/pmcg/p${pipe}_pass$i.log 2>&1 || exit $?
  done
done
find gpurun_out/pmcg -name '*counter_collection*'
