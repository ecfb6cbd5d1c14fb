#!/bin/bash
# Round-6 profile recipe (the round-5 recipe on the round-6 build) (GPU box, repo root).  Kernel-trace stats of Local (C2/C3), C4 and C5
# (2048 envs: one launch, and three launches with DDRL_GNN_TAIL=0); per workload one PMC pass per
# TCC counter (FETCH_SIZE / WRITE_SIZE do not fit one pass) and one of the matrix-core / clock
# counters, all with --kernel-trace; one pass of LDS / issue counters for the Local update and the
# C5 gradient launch.  The C5 passes run the bench configuration (2048 envs, T = 200) for one
# epoch (--sgd-iter 1: 12,800 steps).  Summary:
#   gpurun_out/prof6/pmc_summary.json (tools/pmc_summary.py over the raw passes in /tmp/prof6)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
# raw counter / trace CSVs stay in /tmp (hundreds of MB); the summary, the kernel stats and the
# logs go to gpurun_out/prof6
OUT=/tmp/prof6
KEEP=$R/gpurun_out/prof6
mkdir -p $OUT $KEEP
cd /tmp && export TMPDIR=/tmp
LOCAL="--steps 1 --warmup 0 --no-cpu-baseline --no-pcie"
C4="--env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 0 --no-cpu-baseline --no-pcie"
C5="--env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --sgd-iter 1 --steps 1 --warmup 0 --no-cpu-baseline --no-pcie"
trace() {   # name, bench args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- python3 $R/bench.py "$@" > $OUT/$name.log 2>&1 || return 1
  cp /tmp/prof_$name/run_kernel_stats.csv $KEEP/${name}_kernel_stats.csv
}
pmc() {     # name, tag, "counters", bench args...
  local name=$1 tag=$2 ctr=$3; shift 3
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_${name}_$tag -o run -- python3 $R/bench.py "$@" > $OUT/pmc_${name}_$tag.log 2>&1
}
MF="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
LDS="SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY"
for c in MFMA FETCH_SIZE WRITE_SIZE; do
  ctr=$c; [ $c = MFMA ] && ctr="$MF"
  pmc local $c "$ctr" $LOCAL || exit 1
  pmc c4 $c "$ctr" $C4 || exit 1
  pmc c5 $c "$ctr" $C5 || exit 1
  DDRL_GNN_TAIL=0 pmc c5_3launch $c "$ctr" $C5 || exit 1
done
timeout -s KILL 300 rocprofv3 --pmc $LDS --kernel-trace --output-format csv -d $OUT/lds_local -o run -- python3 $R/bench.py $LOCAL > $OUT/lds_local.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc $LDS --kernel-trace --output-format csv -d $OUT/lds_c5 -o run -- python3 $R/bench.py $C5 > $OUT/lds_c5.log 2>&1 || exit 1
trace local --steps 2 --warmup 1 --no-cpu-baseline --no-pcie || exit 1
trace c4 --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie || exit 1
trace c5 --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-pcie --no-cpu-baseline || exit 1
DDRL_GNN_TAIL=0 trace c5_3launch --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --sgd-iter 1 --steps 1 --warmup 1 --no-pcie --no-cpu-baseline || exit 1
cd $R
python3 tools/pmc_summary.py $OUT > $KEEP/pmc_summary.json || exit 1
cp $OUT/*.log $KEEP/
echo profile done
