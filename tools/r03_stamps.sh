set -o pipefail
mkdir -p gpurun_out/st
DDRL_STAMPS_LIB=1 timeout -k 10 200 python -u tools/diag_stamps.py 4096 > gpurun_out/st/stamps.log 2>&1
echo "rc=$?" >> gpurun_out/st/stamps.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_longhorizon.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/st/lh.log 2>&1
echo "rc=$?" >> gpurun_out/st/lh.log
