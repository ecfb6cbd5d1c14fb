#!/bin/bash
# Rollout fragment as a HIP graph: its bit-identity test first, then the GPU suite, then the
# Local bench A/B (DDRL_ROLLOUT_GRAPH 1 vs 0, twice) and the default bench.
set -e
mkdir -p gpurun_out/graph
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout_graph.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/graph/graph_test.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/graph/tests.log 2>&1
for g in 1 0 1 0; do
  DDRL_ROLLOUT_GRAPH=$g timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/graph/bench_$g.log 2>&1
  grep '^{' gpurun_out/graph/bench_$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph', $g, d['value'], d['ms_per_step'], d['update_kernel_ms'])" | tee -a gpurun_out/graph/ab.txt
done
timeout -k 10 400 python3 bench.py > gpurun_out/graph/bench.log 2>&1
