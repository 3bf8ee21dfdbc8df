# usage: bash scripts/gpu_pmc_attn.sh TAG — counter passes over the three fused attention passes
# alone (attn_bwd_bench.py, C3 encoder shape, dropout 0.1 with keep bits); summary in
# gpurun_out/pmca_TAG/summary_attn.txt.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmca_$1
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAVES"
n=0
for C in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'attn_' --output-format csv -d $O -o attn_p$n -- python scripts/attn_bwd_bench.py > $O/attn_p$n.log 2>&1 || { echo "FAILED pass $n"; tail -5 $O/attn_p$n.log; [ $n -eq 3 ] || exit 1; }
done
python3 scripts/pmc_summary.py $O/attn_p*_counter_collection.csv > $O/summary_attn.txt
head -80 $O/summary_attn.txt
