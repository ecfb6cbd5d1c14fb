#!/bin/bash
# Round-end rehearsal (GPU box, repo root): the whole GPU suite, smoke(), the default bench.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/full_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/full_smoke.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/full_bench.log 2>&1
# the shared-policy lines (C4 SharedDecentral, C5 Graph at 2048 envs), one iteration each
timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/full_bench_c4.log 2>&1
timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/full_bench_c5.log 2>&1
