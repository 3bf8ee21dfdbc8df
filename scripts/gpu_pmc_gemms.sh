# usage: bash scripts/gpu_pmc_gemms.sh TAG — SQ counter passes (one group per run) over the C3 bench's
# N <= 512 input-gradient GEMMs, small-tile GEMMs and the grouped weight gradient (eager steps).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcg_$1
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
n=0
for C in "$P1" "$P2"; do
  n=$((n+1))
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex 'gemm_k128|gemm_grouped|gemm_bf16_lds' --output-format csv -d $O -o g_p$n -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dp-rehearsal --eager > $O/g_p$n.log 2>&1 || { echo "FAILED pass $n"; tail -5 $O/g_p$n.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/g_p*_counter_collection.csv > $O/summary_gemms.txt
grep "==\|MFMA busy\|bank conflict /" $O/summary_gemms.txt
