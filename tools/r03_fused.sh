#!/bin/bash
# GNN fused reduce + Adam step: GNN GPU tests, C5 A/B (fused vs three-launch), then the
# round-end rehearsal (tools/full_check.sh).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn_fused.py tests/test_gpu_gnn.py tests/test_gpu_gnn_layers.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/fused_tests.log 2>&1
for mode in 1 0 1 0; do
  DDRL_GNN_FUSED_ADAM=$mode timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/c5_fused_$mode.log 2>&1
  grep '^{' gpurun_out/c5_fused_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused', $mode, d['value'], d.get('ppo_update_ms_per_minibatch_latency'))" | tee -a gpurun_out/c5_ab.txt
done
bash tools/full_check.sh
