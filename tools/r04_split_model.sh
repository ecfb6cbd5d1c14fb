#!/bin/bash
# r04: cost model of a four-way row split, measured on the two-way kernel:
# timing-only builds that halve the weight-gradient K (DDRL_ABL_HALF_DW: the MFMA work a 32-row
# share saves) and that read the partner's outbox twice more, one read after the other
# (DDRL_ABL_XCHG3: the two more partners' reads a four-way split adds), or load two more
# outboxes with every poll of the first (DDRL_ABL_XCHG3P: the three partners' reads in flight
# together), C4 and Local, two rounds.   VARIANTS="base half_dw ..." OUT=gpurun_out/split
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${OUT:-gpurun_out/split}
mkdir -p $O
for i in 1 2; do
  for v in ${VARIANTS:-base half_dw xchg3 half_dw_xchg3}; do
    timeout -k 10 120 python tools/ablate.py one $R/ddrl_amd/libddrl_hip_abl_$v.so 1024 QuantrupedMultiEnv_SharedDecentral 2>/dev/null | sed "s/^/C4 $v run $i: /" >> $O/timing.log || exit 1
    timeout -k 10 120 python tools/ablate.py one $R/ddrl_amd/libddrl_hip_abl_$v.so 4096 2>/dev/null | sed "s/^/Local $v run $i: /" >> $O/timing.log || exit 1
  done
done
