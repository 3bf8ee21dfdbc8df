# usage: bash scripts/attn_probe.sh — attention bwd microbench under a sweep of EA_ATTN_DBG skip bits (timing probe builds only)
cd $GRAFT_REPO_ROOT
for d in 0 1 2 4 8 16 32 63 0; do echo "dbg=$d: $(EA_ATTN_DBG=$d timeout -k 10 120 python scripts/attn_bwd_bench.py 2>&1 | grep bwd)" || exit 1; done
