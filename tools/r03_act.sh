#!/bin/bash
# Rollout forward with its input loads ahead of the weight staging: GPU suite, kernel trace
# of the Local bench, default bench.
set -e
R=$(pwd)
mkdir -p gpurun_out/act
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/act/tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_local -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $R/gpurun_out/act/trace_local.log 2>&1
cp /tmp/prof_local/run_kernel_stats.csv $R/gpurun_out/act/local_kernel_stats.csv
cd $R
timeout -k 10 400 python3 bench.py > gpurun_out/act/bench.log 2>&1
