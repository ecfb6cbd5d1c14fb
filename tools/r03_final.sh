#!/bin/bash
# Final r03 evidence (GPU box, repo root): smoke(), the C4 / C5 bench lines, and kernel traces
# of the Local bench and of C5 with the final build.
set -e
R=$(pwd)
mkdir -p gpurun_out/final
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/final/bench_c4.log 2>&1
timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/final/bench_c5.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_local -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > $R/gpurun_out/final/trace_local.log 2>&1
cp /tmp/prof_local/run_kernel_stats.csv $R/gpurun_out/final/local_kernel_stats.csv
