#!/bin/bash
# decode timing: skinny GEMM on/off, then a kernel-trace summary of the default
set -o pipefail
OUT=gpurun_out/dec_${1:-a}
mkdir -p $OUT
export TMPDIR=/tmp
true &&
true &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o dec -- python3 scripts/decode_bench.py --utts 2 > $OUT/prof.log 2>&1
rc=$?
find $OUT/prof -name '*kernel_stats.csv' -exec cp {} $OUT/kernel_stats.csv \;
exit $rc
