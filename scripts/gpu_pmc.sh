# usage: bash scripts/gpu_pmc.sh <tag>  — HBM traffic (FETCH_SIZE, WRITE_SIZE: separate passes) of
# the roofline kernel (conv2 forward implicit GEMM) over a short eager bench run, summarised
# into gpurun_out/pmc/pmc_conv2_fwd.json (copy to profiles/ to make bench.py report it).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
mkdir -p gpurun_out/pmc
RX='gemm_(pipe<true, true, 1, 256(, 4)?>|bf16_lds<256, 256, 4, true, true, 2, 1>)'
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc -o ${TAG}_fetch -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dp-rehearsal --eager > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc -o ${TAG}_write -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-dp-rehearsal --eager > gpurun_out/pmc_write.log 2>&1 || exit $?
python scripts/pmc_to_json.py gpurun_out/pmc/${TAG}_fetch_counter_collection.csv gpurun_out/pmc/${TAG}_write_counter_collection.csv gpurun_out/pmc/pmc_conv2_fwd.json
