#!/bin/bash
# Round-3 profile recipe (GPU box, repo root): kernel-trace stats of the Local (C2/C3), C4
# SharedDecentral and C5 Graph (2048 envs) workloads, then one PMC pass per TCC counter
# (FETCH_SIZE / WRITE_SIZE do not fit one pass) for each workload; C5's PMC passes run at
# 128 envs (8,000 minibatch steps; the per-step traffic does not depend on the env count).
# Trace directories stay in /tmp; summaries go to gpurun_out/prof.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
trace() {   # name, bench args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $OUT/$name.log 2>&1
  cp /tmp/prof_$name/run_kernel_stats.csv $OUT/${name}_kernel_stats.csv
}
pmc() {     # name, counter, bench args...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $OUT/pmc_${name}_$ctr -o run -- python3 $R/bench.py "$@" > $OUT/pmc_${name}_$ctr.log 2>&1
}
trace local --steps 2 --warmup 1 --no-cpu-baseline --no-pcie
trace c4 --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie
trace c5 --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-pcie
for c in FETCH_SIZE WRITE_SIZE; do
  pmc local $c --steps 1 --warmup 0 --no-cpu-baseline --no-pcie
  pmc c4 $c --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 0 --no-cpu-baseline --no-pcie
  pmc c5 $c --env QuantrupedMultiEnv_DecentralShared_Graph --envs 128 --steps 1 --warmup 0 --no-pcie
done
cd $R
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json
DDRL_STAMPS_LIB=1 timeout -k 10 200 python3 tools/diag_stamps.py 4096 > $OUT/stamps.log 2>&1
