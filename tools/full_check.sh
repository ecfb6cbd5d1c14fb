#!/bin/bash
# Round-end rehearsal (GPU box, repo root): the whole GPU suite, smoke(), the default bench.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/full_bench.log 2>&1
