#!/bin/bash
# r04: the data-parallel learner at one rank (RCCL communicator of one, DDRL_FORCE_DDP=1): C4
# SharedDecentral at 4096 envs and C5 Graph at 2048 envs, native loop, split mode; then the
# per-kernel times of the C4 step under rocprofv3 (512 envs).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ddp4
mkdir -p $O
export MASTER_ADDR=127.0.0.1 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 DDRL_FORCE_DDP=1
MASTER_PORT=29521 timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie --ddp-mode split > $O/bench_c4_ddp1.log 2>&1 || exit 1
MASTER_PORT=29522 timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie --ddp-mode split > $O/bench_c5_ddp1.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
MASTER_PORT=29523 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_ddp4 -o run -- python3 $R/bench.py --env QuantrupedMultiEnv_SharedDecentral --envs 512 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie --ddp-mode split > $O/trace_c4_ddp1_512.log 2>&1 || exit 1
cp /tmp/prof_ddp4/run_kernel_stats.csv $O/c4_ddp1_512_kernel_stats.csv
