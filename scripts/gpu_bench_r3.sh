# usage: bash scripts/gpu_bench_r3.sh TAG — the default bench line (C3, N=1, with the CPU baseline)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bench_$1
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
