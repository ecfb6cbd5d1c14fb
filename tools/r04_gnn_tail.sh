#!/bin/bash
# r04: the one-launch GNN step -- its GNN tests, the C5 bench lines (one launch with nt / plain
# partial stores, three launches), the phase timeline.
set -o pipefail
mkdir -p gpurun_out/gt
timeout -k 10 600 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_gnn_rollback.py tests/test_gpu_ddp_native.py tests/test_gpu_gnn_layers.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gt/tests.log 2>&1 || exit 1
B="--env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie"
timeout -k 10 300 python3 bench.py $B > gpurun_out/gt/bench_c5.log 2>&1 || exit 1
DDRL_LIB=libddrl_hip_gl2.so timeout -k 10 300 python3 bench.py $B > gpurun_out/gt/bench_c5_gl2.log 2>&1 || exit 1
DDRL_GNN_TAIL=0 timeout -k 10 300 python3 bench.py $B > gpurun_out/gt/bench_c5_3launch.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py $B > gpurun_out/gt/bench_c5_b.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/diag_gnn_stamps.py 2048 mpnn > gpurun_out/gt/stamps_mpnn.log 2>&1 || exit 1
# fcnet forward: layer-1 tanh interleaved into layer 2's MFMAs (default) vs all before them
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "update or schedule or rollout" > gpurun_out/gt/parity.log 2>&1 || exit 1
for i in 1 2; do
  for v in libddrl_hip.so libddrl_hip_fwd0.so; do
    timeout -k 10 100 python tools/ablate.py one $(pwd)/ddrl_amd/$v 4096 2>/dev/null | sed "s/^/$v run $i: /" >> gpurun_out/gt/fwd_ab.log || exit 1
  done
done
