# Round 5 (a): VGPR-form MFMA build (libespnet_amd_vf.so) vs the default build, on the N = 512
# GEMM shapes (scripts/gemm_n512.py, incl. gemm_k128 and hipBLASLt) and on the C3 step with
# hipBLASLt on / off (EA_GEMM_BLASLT=1 / 0), alternated twice.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
for L in libespnet_amd.so libespnet_amd_vf.so; do
  echo "== $L" >> $O/gemm.txt
  EA_LIB_NAME=$L timeout -k 10 240 python -u scripts/gemm_n512.py >> $O/gemm.txt 2>&1 || exit 1
done
for r in 1 2; do
  for L in libespnet_amd.so libespnet_amd_vf.so; do
    for b in 1 0; do
      EA_LIB_NAME=$L EA_GEMM_BLASLT=$b timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-dp-rehearsal > $O/b_${L}_${b}_$r.json 2> $O/b_${L}_${b}_$r.err || exit 1
      python3 -c "import json; d=json.load(open('$O/b_${L}_${b}_$r.json')); print('$L blaslt=$b', d['value'], d['step_ms_median'])" | tee -a $O/bench.txt
    done
  done
done
