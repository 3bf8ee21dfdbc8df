# PMC of the shipped (pipelined) fused attention kernels: attn_fwd2 / attn_bwdq2 / attn_bwdkv2 at
# the C3 encoder shape (attn_bwd_bench.py, p = 0.1); one counter group per run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc_attn_r4
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for i in 1 2 3; do
  eval C=\$P$i
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex 'attn_' --output-format csv -d $O -o attn_p$i -- python scripts/attn_bwd_bench.py > $O/attn_p$i.log 2>&1 || { echo "FAILED p$i"; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'attn_' --output-format csv -d $O -o attn_fetch -- python scripts/attn_bwd_bench.py > $O/attn_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'attn_' --output-format csv -d $O -o attn_write -- python scripts/attn_bwd_bench.py > $O/attn_write.log 2>&1 || exit 1
python scripts/pmc_summary.py $O/attn_p1_counter_collection.csv $O/attn_p2_counter_collection.csv $O/attn_p3_counter_collection.csv $O/attn_fetch_counter_collection.csv $O/attn_write_counter_collection.csv > $O/summary.txt 2>&1
grep -v "^   [A-Z]" $O/summary.txt | head -40
