#!/bin/bash
# A/B of one environment switch on the C3 bench, alternated, plus a kernel trace per value.
#   scripts/ab_env.sh OUTDIR VAR "v1 v2 ..." [ROUNDS]     (DP=1 in the environment: with the
#   bench's DP-rehearsal leg, whose step time is printed too)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; VAR=$2; VALS=$3; R=${4:-2}
ARGS="--no-cpu-baseline"; [ "${DP:-0}" = 1 ] || ARGS="$ARGS --no-dp-rehearsal"
mkdir -p "$O"
for r in $(seq 1 $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 $ARGS > "$O/bench_${v}_$r.log" 2>&1 || { echo "bench $v failed"; tail -20 "$O/bench_${v}_$r.log"; exit 1; }
    python3 -c "import json,sys; l=[x for x in open('$O/bench_${v}_$r.log') if x.startswith('{')][-1]; d=json.loads(l); dp=d.get('dp_rehearsal'); print('$VAR=$v', d['value'], d['ms_per_step'], '' if dp is None else 'dp %s %s' % (dp['value'], dp['ms_per_step']))"
  done
done
for v in $VALS; do
  export $VAR=$v
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/tr_$v" -o t -- python -u bench.py --steps 5 --warmup 4 $ARGS --dp-rehearsal-steps 6 > "$O/trace_$v.log" 2>&1 || { echo "trace $v failed"; exit 1; }
done
echo done
