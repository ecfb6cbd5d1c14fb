set -o pipefail
mkdir -p gpurun_out/chk
bash tools/r03_time.sh cur ht
DDRL_STAMPS_LIB=1 timeout -k 10 200 python -u tools/diag_stamps.py 4096 > gpurun_out/chk/stamps.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cup.py tests/test_gpu_rollback.py tests/test_gpu_bounds.py tests/test_gpu_longhorizon.py tests/test_gpu_gnn.py tests/test_gpu_ddp_native.py tests/test_gpu_golden.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/chk/tests.log 2>&1
echo "rc=$?" >> gpurun_out/chk/tests.log
