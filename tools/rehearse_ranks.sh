#!/bin/bash
# Two ranks on the one GPU of a test box over gloo (DDRL_DIST_BACKEND=gloo): the replica
# path (Local) and the data-parallel path (C4, Python loop over gloo), short runs.
set -e
mkdir -p gpurun_out
export DDRL_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 \
  bench.py --gpus 2 --envs 1024 --steps 2 --warmup 1 > gpurun_out/rehearse_local.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29522 \
  bench.py --gpus 2 --env QuantrupedMultiEnv_SharedDecentral --envs 256 --steps 1 --warmup 1 > gpurun_out/rehearse_c4.log 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 \
  bench.py --gpus 2 --env QuantrupedMultiEnv_DecentralShared_Graph --envs 128 --steps 1 --warmup 1 > gpurun_out/rehearse_c5.log 2>&1
# the default N=1 line under torchrun as the driver launches it (RCCL process group of one rank)
unset DDRL_DIST_BACKEND
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29524 \
  bench.py --gpus 1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/rehearse_n1.log 2>&1
