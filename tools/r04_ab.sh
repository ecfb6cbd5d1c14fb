#!/bin/bash
# r04 A/B of in-tree builds: the update tests on the default library (TESTS=0 skips them), then
# us per sequential update step of each ddrl_amd/<lib> given, Local 4096 and C4 1024, 2 rounds.
#   bash tools/r04_ab.sh libddrl_hip.so libddrl_hip_lxe0.so      (OUT=gpurun_out/ab4)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=${OUT:-gpurun_out/ab4}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py tests/test_gpu_rollback.py tests/test_gpu_golden.py tests/test_gpu_checkpoint.py tests/test_gpu_cup.py tests/test_gpu_fullsize.py tests/test_gpu_bounds.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
fi
for i in 1 2; do
  for v in "$@"; do
    timeout -k 10 120 python tools/ablate.py one $R/ddrl_amd/$v 4096 2>/dev/null | sed "s/^/Local $v run $i: /" >> $O/timing.log || exit 1
    timeout -k 10 120 python tools/ablate.py one $R/ddrl_amd/$v 1024 QuantrupedMultiEnv_SharedDecentral 2>/dev/null | sed "s/^/C4 $v run $i: /" >> $O/timing.log || exit 1
  done
done
