# Round 5 attention VALU diet: attention / model tests, then the C3 bench under a kernel trace
# (per-kernel averages of the three attention passes in scripts/step_anatomy.py's table).
# usage: bash scripts/gpu_attn_r5.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/attn_$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_attention_gpu.py \
  tests/test_model_gpu.py tests/test_inference_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['step_ms_median'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o prof -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-dp-rehearsal > $O/prof.json 2> $O/prof.err || exit 1
python3 scripts/step_anatomy.py $O/prof_kernel_trace.csv > $O/anatomy.txt
grep -i "attn" $O/prof_kernel_stats.csv | cut -d, -f1-8 | head -20
