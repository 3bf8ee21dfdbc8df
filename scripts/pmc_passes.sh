#!/bin/bash
# Counter passes for the kernels matching REGEX while CMD runs: three SQ / TCC groups and the
# FETCH_SIZE / WRITE_SIZE traffic passes, each its own rocprofv3 run with --kernel-trace only
# (MI355X_MICROARCH.md § HBM / rocprofv3), then scripts/pmc_summary.py over them.
#   scripts/pmc_passes.sh OUTDIR NAME REGEX CMD...      (summary: OUTDIR/summary_NAME.txt)
set -o pipefail
export TMPDIR=/tmp
O=$1; NAME=$2; RX=$3; shift 3
mkdir -p "$O"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for p in 1 2 3 fetch write; do
  case $p in
    1) C=$P1 ;; 2) C=$P2 ;; 3) C=$P3 ;; fetch) C=FETCH_SIZE ;; write) C=WRITE_SIZE ;;
  esac
  timeout -s KILL 150 rocprofv3 --pmc $C --kernel-include-regex "$RX" --output-format csv -d "$O" -o "${NAME}_$p" \
    -- "$@" > "$O/${NAME}_$p.log" 2>&1 || { echo "pass $p failed"; exit 1; }
done
python3 scripts/pmc_summary.py "$O"/${NAME}_*_counter_collection.csv > "$O/summary_${NAME}.txt"
cat "$O/summary_${NAME}.txt"
