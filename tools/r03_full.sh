set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/full/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full/smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/full/bench.log 2>&1
