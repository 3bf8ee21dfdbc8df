set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/diag
timeout -k 10 500 python -u scripts/diag/spawn_diag.py > gpurun_out/diag/spawn.log 2>&1; rc=$?
grep -E "^bs|Error|error" gpurun_out/diag/spawn.log | head -40; exit $rc
