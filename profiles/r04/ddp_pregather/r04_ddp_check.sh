set -o pipefail
mkdir -p gpurun_out/ddp4
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp_native.py tests/test_gpu_rollback.py tests/test_gpu_bounds.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ddp4/tests.log 2>&1 || exit 1
bash tools/r04_ddp.sh
