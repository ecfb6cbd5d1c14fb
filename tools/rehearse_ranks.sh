#!/bin/bash
# Multi-rank rehearsal of bench.py on the one GPU of a test box: N ranks over
# gloo (DDRL_DIST_BACKEND=gloo, every rank on device 0), N = ${RANKS:-"4 8"}:
#   Local replicas (the driver's default SCALE line), C4 in the default shared-policy mode
#   (gather), C4 through the split-mode data-parallel learner (Python loop over gloo, one epoch),
#   C5 gather; then the N=1 line under torchrun as the driver launches it (RCCL group of one).
# Every step has its own time limit and the steps are chained: the first failure ends the script.
set -e
mkdir -p gpurun_out/rehearse
export DDRL_DIST_BACKEND=gloo
port=29600
run() {   # run <ranks> <log> <bench args...>
  local n=$1 log=$2
  shift 2
  port=$((port + 1))
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus "$n" "$@" > "gpurun_out/rehearse/$log" 2>&1
  tail -n 1 "gpurun_out/rehearse/$log"
}
for n in ${RANKS:-4 8}; do
  run "$n" "local_w$n.log" --envs 4096 --steps 2 --warmup 1
  run "$n" "c4_gather_w$n.log" --env QuantrupedMultiEnv_SharedDecentral --envs 1024 --steps 1 --warmup 1
  run "$n" "c4_ddp_split_w$n.log" --env QuantrupedMultiEnv_SharedDecentral --envs 256 --steps 1 --warmup 1 \
    --shared-mode ddp --ddp-mode split --sgd-iter 1
  # ranks sharing one GPU cannot all hold the one-launch GNN step's 256-block grid resident (its
  # waits would end at their 3 s bound; the bench then reruns the update on three launches), so
  # the shared-GPU rehearsal runs the three-launch step; on the 8-GPU node every rank has a GPU
  DDRL_GNN_TAIL=0 run "$n" "c5_gather_w$n.log" --env QuantrupedMultiEnv_DecentralShared_Graph --envs 256 --steps 1 --warmup 1
done
unset DDRL_DIST_BACKEND
run 1 n1_torchrun.log --steps 2 --warmup 1 --no-cpu-baseline
