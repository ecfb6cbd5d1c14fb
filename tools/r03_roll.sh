#!/bin/bash
# Rollout kernels (chunked filter push, predicated reward loads, batched GAE) + the relaxed
# fused GNN step: GPU suite, C5 A/B (DDRL_GNN_FUSED_ADAM 2 vs 0), Local bench, kernel trace.
set -e
R=$(pwd)
mkdir -p gpurun_out/roll
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/roll/tests.log 2>&1
for mode in 2 0 2 0; do
  DDRL_GNN_FUSED_ADAM=$mode timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/roll/c5_$mode.log 2>&1
  grep '^{' gpurun_out/roll/c5_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused', $mode, d['value'], d.get('ppo_update_ms_per_minibatch_latency'))" | tee -a gpurun_out/roll/c5_ab.txt
done
timeout -k 10 400 python3 bench.py > gpurun_out/roll/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_local -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $R/gpurun_out/roll/trace_local.log 2>&1
cp /tmp/prof_local/run_kernel_stats.csv $R/gpurun_out/roll/local_kernel_stats.csv
