# PMC: 7968x512x2048 on the 64x128 tile, on gemm_k128, and hipBLASLt; kernel trace of the decode bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
run() {  # name cmd...
  local name=$1 ctr=$2
  shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O -o $name -- "$@" > $O/$name.log 2>&1 || { echo "FAILED $name"; exit 1; }
  echo "ok $name"
}
for i in 1 2 3; do
  eval C=\$P$i
  run lds64_p$i "$C" python scripts/gemm_one.py 7968 512 2048 1 1 10
  EA_GEMM_K128=3 run k128_p$i "$C" python scripts/gemm_one.py 7968 512 2048 1 1 10
  run blas_p$i "$C" python scripts/blaslt_one.py 7968 512 2048 10
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o dec -- python scripts/decode_bench.py --utts 2 > $O/dec.log 2>&1 || exit 1
ls $O
