# usage: bash scripts/gpu_pmc_r5.sh TAG — counter passes (one counter group per run, kernel-trace
# only) for the 256x256 ping-pong GEMM family: the FFN GEMMs with their epilogues and a square
# 4096^3 product (gemm_ffn_one.py), the conv2 implicit GEMMs (sub_bench.py, serial streams), and
# the attention passes (attn_bwd_bench.py).  Results under gpurun_out/pmc5_TAG/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
O=gpurun_out/pmc5_$T
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
run() {  # name regex counters cmd...
  local name=$1 rx=$2 ctr=$3
  shift 3
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $O -o $name -- "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; exit 1; }
  echo "ok $name"
}
for i in 1 2 3; do
  eval C=\$P$i
  run ffn_p$i 'gemm_' "$C" python scripts/gemm_ffn_one.py 5
  run conv_p$i 'gemm_pipe' "$C" python scripts/sub_bench.py 3
  run attn_p$i 'attn_' "$C" python scripts/attn_bwd_bench.py
done
run ffn_fetch 'gemm_' FETCH_SIZE python scripts/gemm_ffn_one.py 5
run ffn_write 'gemm_' WRITE_SIZE python scripts/gemm_ffn_one.py 5
run conv_fetch 'gemm_pipe' FETCH_SIZE python scripts/sub_bench.py 3
run conv_write 'gemm_pipe' WRITE_SIZE python scripts/sub_bench.py 3
python3 scripts/pmc_summary.py $O/ffn_*_counter_collection.csv > $O/summary_ffn.txt
python3 scripts/pmc_summary.py $O/conv_*_counter_collection.csv > $O/summary_conv.txt
python3 scripts/pmc_summary.py $O/attn_*_counter_collection.csv > $O/summary_attn.txt
ls $O
