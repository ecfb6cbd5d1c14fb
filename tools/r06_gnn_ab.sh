#!/bin/bash
# r06: C5 bench lines (2048 envs, one-launch GNN step) of the default library and of the in-tree
# variant builds named on the command line (DDRL_LIB), two rounds each; prints us per step.
set -o pipefail
O=gpurun_out/r06/gab
mkdir -p $O
B5="--env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie"
for i in 1 2; do
  timeout -k 10 300 python3 bench.py $B5 > $O/default_$i.log 2>&1 || exit 1
  for v in "$@"; do
    DDRL_LIB=$(pwd)/ddrl_amd/libddrl_hip_abl_$v.so timeout -k 10 300 python3 bench.py $B5 > $O/${v}_$i.log 2>&1 || exit 1
  done
done
python3 - "$@" <<'PY'
import json, sys
for v in ["default"] + sys.argv[1:]:
    us = [json.loads(open(f"gpurun_out/r06/gab/{v}_{i}.log").read().strip().splitlines()[-1])["ppo_update_ms_per_minibatch_latency"] * 1e3 for i in (1, 2)]
    print(v, " ".join(f"{u:.3f}" for u in us), "us/step")
PY
