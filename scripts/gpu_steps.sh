#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit, logging to
# gpurun_out/<dir>/NN.log.  A step that fails its checks (exit 1) does not stop the run; a
# fault, abort, segfault or time limit (124 / 134 / 137 / 139 / negative) does: nothing more
# is started on the GPU after it.
#   scripts/gpu_steps.sh DIR SECONDS "cmd 1" "cmd 2" ...
set -u
dir=gpurun_out/$1; lim=$2; shift 2
mkdir -p "$dir"
i=0; worst=0
for cmd in "$@"; do
  i=$((i + 1)); log=$(printf "%s/%02d.log" "$dir" "$i")
  echo "== [$i] $cmd" | tee "$log"
  start=$(date +%s)
  timeout -k 10 "$lim" bash -c "$cmd" >> "$log" 2>&1
  rc=$?
  echo "== [$i] exit $rc after $(( $(date +%s) - start )) s" | tee -a "$log"
  tail -n 6 "$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping: exit $rc"; exit $rc
  fi
  [ $rc -ne 0 ] && worst=$rc
done
exit $worst
