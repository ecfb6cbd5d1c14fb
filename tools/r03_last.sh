#!/bin/bash
# Round-end check of the final tree: GPU suite, smoke, default bench.
set -e
mkdir -p gpurun_out/last
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/last/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/last/smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/last/bench.log 2>&1
