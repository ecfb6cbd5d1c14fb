set -o pipefail
mkdir -p gpurun_out/r03base
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03base/gpu_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r03base/bench.log 2>&1 &&
DDRL_STAMPS_LIB=1 timeout -k 10 200 python -u tools/diag_stamps.py 512 > gpurun_out/r03base/stamps.log 2>&1
