set -o pipefail
mkdir -p gpurun_out/gnn
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn_layers.py tests/test_gpu_gnn.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gnn/tests.log 2>&1
