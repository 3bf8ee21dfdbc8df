set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/dpcap
EA_STREAM_WGRAD=0 timeout -k 10 150 python -u -m pytest tests/test_dp_capture_gpu.py -x -v -s --timeout 140 --timeout-method thread -k rccl > gpurun_out/dpcap/s0.log 2>&1; echo "s0 rc=$?"; tail -5 gpurun_out/dpcap/s0.log
timeout -k 10 150 python -u -m pytest tests/test_dp_capture_gpu.py -x -v -s --timeout 140 --timeout-method thread -k rccl > gpurun_out/dpcap/s1.log 2>&1; echo "s1 rc=$?"; tail -30 gpurun_out/dpcap/s1.log
