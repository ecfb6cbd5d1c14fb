#!/bin/bash
# Kernel-trace stats of the data-parallel learner at one rank (C4, 512 envs, split mode):
# the library loop (ddrl_ppo_update_ddp) and the Python loop, each under rocprofv3 with the
# process group set up from env variables (no launcher between the profiler and python).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_ddp
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 DDRL_FORCE_DDP=1
for loop in native python; do
  DDRL_DDP_LOOP=$loop timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ddp_$loop -o run -- \
    python3 $R/bench.py --env QuantrupedMultiEnv_SharedDecentral --envs 512 --steps 1 --warmup 1 \
    --no-cpu-baseline --no-pcie --ddp-mode split > $OUT/ddp_$loop.log 2>&1
  cp /tmp/prof_ddp_$loop/run_kernel_stats.csv $OUT/ddp_${loop}_kernel_stats.csv
done
