#!/bin/bash
# r04: the GNN tests on the default library, then C5 bench lines (2048 envs) of the default and
# of the in-tree baseline build named by $1 (DDRL_LIB), two rounds each.
set -o pipefail
O=gpurun_out/gab
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_gnn_layers.py tests/test_gpu_gnn_rollback.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
B5="--env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $B5 > $O/new_$i.log 2>&1 || exit 1
  DDRL_LIB=$1 timeout -k 10 300 python3 bench.py $B5 > $O/base_$i.log 2>&1 || exit 1
done
