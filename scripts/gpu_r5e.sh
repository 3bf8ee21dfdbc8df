# Round 5 (e): attention tests + counter passes over the attention passes, then the C3 bench
# with EA_JOIN_ONCE 0 / 1 alternated twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_attention_gpu.py tests/test_model_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_attn.sh e > $O/pmc.txt 2>&1 || exit 1
grep -A3 "^== attn_fwd2_kernel<true, 1>\|^== attn_bwdq2_kernel<true, 1>\|^== attn_bwdkv2_kernel<true, 1>" gpurun_out/pmca_e/summary_attn.txt | grep "==\|INSTS_VALU" ; grep "median" gpurun_out/pmca_e/summary_attn.txt
for r in 1 2; do
  for v in 0 1; do
    EA_JOIN_ONCE=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); print('JOIN_ONCE=$v', d['value'], d['step_ms_median'])" | tee -a $O/bench.txt
  done
done
