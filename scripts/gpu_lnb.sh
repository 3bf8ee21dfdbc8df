# LayerNorm backward variants (scripts/ln_bwd_bench.py): waves per block x rows per block
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lnb
for v in "4 16" "8 16" "4 8" "8 32" "4 16"; do set -- $v
  echo "W=$1 RPB=$2"
  EA_LN_BWD_W=$1 EA_LN_BWD_RPB=$2 timeout -k 10 120 python scripts/ln_bwd_bench.py 2>/dev/null || exit 1
done 2>&1 | tee gpurun_out/lnb/out2.txt
