#!/bin/bash
# Two-launch filter push + GAE prefetch depth: GPU suite, Local bench, kernel trace.
set -e
R=$(pwd)
mkdir -p gpurun_out/roll2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/roll2/tests.log 2>&1
timeout -k 10 400 python3 bench.py > gpurun_out/roll2/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_local -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $R/gpurun_out/roll2/trace_local.log 2>&1
cp /tmp/prof_local/run_kernel_stats.csv $R/gpurun_out/roll2/local_kernel_stats.csv
