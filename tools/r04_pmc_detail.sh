#!/bin/bash
# r04: issue / wait / LDS counters of the Local update kernel (tools/ablate.py one, 512 envs:
# 8,000 steps x 4 policies) and of the C5 GNN launch (bench, 128 envs), two SQ passes each.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcd
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/local_p$i -o run -- python3 $R/tools/ablate.py one $R/ddrl_amd/libddrl_hip.so 512 > $OUT/local_p$i.log 2>&1 || exit 1
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/c5_p$i -o run -- python3 $R/bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 128 --steps 1 --warmup 0 --no-pcie --no-cpu-baseline > $OUT/c5_p$i.log 2>&1 || exit 1
done
