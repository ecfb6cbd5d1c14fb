#!/bin/bash
# Round-1 profile recipe (run on the GPU box from the repo root):
#   kernel-trace stats of the default bench (Local, C2/C3 workload), then one PMC pass per TCC
#   counter (FETCH_SIZE and WRITE_SIZE do not fit one pass), then kernel-trace stats of the
#   shared-policy (C4) and GraphNet (C5, 2048 envs) workloads, then the default bench with the
#   CPU baseline.  Trace directories stay in /tmp (the C5 kernel trace alone is >100 MB); only
#   the summaries are copied to gpurun_out/prof.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
trace() {   # name, bench args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $OUT/$name.log 2>&1
  cp /tmp/prof_$name/run_kernel_stats.csv $OUT/${name}_kernel_stats.csv
}
trace trace --steps 2 --warmup 1 --no-cpu-baseline --no-pcie
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pcie > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-pcie > $OUT/pmc_write.log 2>&1
trace c4 --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie
trace c5 --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-pcie
cd $R
# the bench reports traffic from profiles/r01/pmc_update.json: refresh it from these passes
python3 tools/pmc_summary.py $OUT > $OUT/pmc_update.json
cp $OUT/pmc_update.json $R/profiles/r01/pmc_update.json
timeout -k 10 400 python3 bench.py > $OUT/bench_default.log 2>&1
