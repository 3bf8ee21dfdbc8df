# usage: bash scripts/gpu_pmc_r3.sh TAG — counter passes (one pass per run, kernel-trace only) for
# the round-3 perf targets: the fused rel-pos attention (attn_bwd_bench.py, p = 0.1), the N = 512
# Linear GEMMs (7968 x 512 x 2048 forward, 7968 x 512 x 512, 7968 x 2048 x 512) and the conv2
# implicit GEMMs (sub_bench.py, serial streams).  Results under gpurun_out/pmc3/.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmc3
mkdir -p $O
T=$1
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
run() {  # name regex pass-counters cmd...
  local name=$1 rx=$2 ctr=$3
  shift 3
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$rx" --output-format csv -d $O -o ${T}_$name -- "$@" > $O/${T}_$name.log 2>&1 || { echo "FAILED $name"; exit 1; }
  echo "ok $name"
}
for i in 1 2 3; do
  eval C=\$P$i
  run attn_p$i 'attn_' "$C" python scripts/attn_bwd_bench.py
done
run attn_fetch 'attn_' FETCH_SIZE python scripts/attn_bwd_bench.py
run attn_write 'attn_' WRITE_SIZE python scripts/attn_bwd_bench.py
for shp in "7968 512 2048 1 1" "7968 512 512 1 1" "7968 2048 512 1 1"; do
  nm=g$(echo $shp | tr ' ' '_')
  for i in 1 2 3; do
    eval C=\$P$i
    run ${nm}_p$i 'gemm_' "$C" python scripts/gemm_one.py $shp 10
  done
  run ${nm}_fetch 'gemm_' FETCH_SIZE python scripts/gemm_one.py $shp 10
done
for i in 1 3; do
  eval C=\$P$i
  run conv_p$i 'gemm_pipe' "$C" python scripts/sub_bench.py 3
done
run conv_fetch 'gemm_pipe' FETCH_SIZE python scripts/sub_bench.py 3
run conv_write 'gemm_pipe' WRITE_SIZE python scripts/sub_bench.py 3
ls $O
