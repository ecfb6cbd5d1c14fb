#!/bin/bash
# Round-4 profile recipe (GPU box, repo root): kernel-trace stats of the Local (C2/C3), C4
# SharedDecentral and C5 Graph (2048 envs) workloads; per workload one PMC pass per TCC counter
# (FETCH_SIZE / WRITE_SIZE do not fit one pass) and one pass of the matrix-core / clock counters
# (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES, GRBM_GUI_ACTIVE) with --kernel-trace,
# so every counter row has its dispatch's duration.  C5's PMC passes run at 128 envs (8,000
# minibatch steps; the per-step figures do not depend on the env count).  Summaries:
#   python3 tools/pmc_summary.py gpurun_out/prof4 > profiles/r04/pmc_summary.json
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof4
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
LOCAL="--steps 1 --warmup 0 --no-cpu-baseline --no-pcie"
C4="--env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 0 --no-cpu-baseline --no-pcie"
C5="--env QuantrupedMultiEnv_DecentralShared_Graph --envs 128 --steps 1 --warmup 0 --no-pcie"
trace() {   # name, bench args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $OUT/$name.log 2>&1 || return 1
  cp /tmp/prof_$name/run_kernel_stats.csv $OUT/${name}_kernel_stats.csv
}
pmc() {     # name, tag, "counters", bench args...
  local name=$1 tag=$2 ctr=$3; shift 3
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_${name}_$tag -o run -- python3 $R/bench.py "$@" > $OUT/pmc_${name}_$tag.log 2>&1
}
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
pmc local MFMA "$MF" $LOCAL || exit 1
pmc c4 MFMA "$MF" $C4 || exit 1
pmc c5 MFMA "$MF" $C5 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  pmc local $c $c $LOCAL || exit 1
  pmc c4 $c $c $C4 || exit 1
  pmc c5 $c $c $C5 || exit 1
done
trace local --steps 2 --warmup 1 --no-cpu-baseline --no-pcie || exit 1
trace c4 --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie || exit 1
trace c5 --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-pcie || exit 1
cd $R
python3 tools/pmc_summary.py $OUT > $OUT/pmc_summary.json || exit 1
