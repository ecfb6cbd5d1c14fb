#!/bin/bash
# r05: one-rank data-parallel step (C4 4096 envs, C5 2048 envs) of the default library and of the
# in-tree variant builds named on the command line (DDRL_LIB), us per step.
set -o pipefail
O=gpurun_out/r05/ddp_ab
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in default "$@"; do
  lib=$(pwd)/ddrl_amd/libddrl_hip.so
  [ "$v" = default ] || lib=$(pwd)/ddrl_amd/libddrl_hip_abl_$v.so
  for e in "QuantrupedMultiEnv_SharedDecentral 4096" "QuantrupedMultiEnv_DecentralShared_Graph 2048"; do
    set -- $e
    DDRL_LIB=$lib DDRL_FORCE_DDP=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --env $1 --envs $2 --steps 1 --warmup 1 --no-cpu-baseline \
      --no-pcie > $O/${v}_$1.log 2>&1 || exit 1
    echo "$v $1 $(grep -o '"ppo_update_ms_per_minibatch_latency": [0-9.]*' $O/${v}_$1.log)"
  done
done
