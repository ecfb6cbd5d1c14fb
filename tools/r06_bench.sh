#!/bin/bash
# r06 bench lines of the other configurations (C4 SharedDecentral 4096 envs, C5 Graph 2048 envs:
# one launch and three launches per step) and the phase stamps of the Local update kernel
# (diagnostic build shipped as ddrl_amd/libddrl_hip_stmp.so).  Each step has its own limit.
set -o pipefail
O=gpurun_out/r06/bench
mkdir -p $O
timeout -k 10 400 python3 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 2 --warmup 1 > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 > $O/bench_c5.log 2>&1 || exit 1
DDRL_GNN_TAIL=0 timeout -k 10 400 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_c5_3launch.log 2>&1 || exit 1
if [ -f ddrl_amd/libddrl_hip_stmp.so ]; then
  DDRL_STAMPS_LIB=libddrl_hip_stmp.so timeout -k 10 300 python tools/diag_stamps.py 4096 > $O/stamps_local4096.log 2>&1 || exit 1
fi
for f in $O/bench_*.log; do echo "$f: $(tail -n 1 $f | cut -c1-160)"; done
