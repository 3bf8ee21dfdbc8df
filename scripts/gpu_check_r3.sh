# usage: bash scripts/gpu_check_r3.sh TAG [pytest files...] — parity tests for the touched kernels,
# attention + conv2 microbenchmarks under rocprofv3 --kernel-trace --stats, then a short bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
shift
O=gpurun_out/chk_$T
mkdir -p $O
FILES=${@:-tests/test_attention_gpu.py tests/test_subsampling_gpu.py tests/test_model_gpu.py tests/test_model_sized_gpu.py}
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $FILES > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o attn -- python scripts/attn_bwd_bench.py > $O/attn.log 2>&1 || exit 1
grep attn_ $O/attn.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o sub -- python scripts/sub_bench.py 5 > $O/sub.log 2>&1 || exit 1
python3 - <<EOF
import csv
for f in ("$O/attn_kernel_stats.csv", "$O/sub_kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        if any(k in r["Name"] for k in ("attn", "gemm_pipe")):
            print(r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Name"][:90])
EOF
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 1
cat $O/bench.json
