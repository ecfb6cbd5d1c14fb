#!/bin/bash
# r05: the whole GPU suite on the padded-LDS default library, then A/B timing against the
# in-tree variant builds named on the command line: Local update us/step (tools/ablate.py one,
# 4096 envs; the state digest shows bit-identity) and the C5 bench line (tools/r05_gnn_ab.sh).
set -o pipefail
O=gpurun_out/r05
mkdir -p $O/ab
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $O/gpu_tests_all.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -4 $O/gpu_tests_all.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/ablate.py one $(pwd)/ddrl_amd/libddrl_hip.so 4096 2>/dev/null | sed "s/^/default run $i: /" >> $O/ab/local.log || exit 1
  for v in "$@"; do
    timeout -k 10 120 python tools/ablate.py one $(pwd)/ddrl_amd/libddrl_hip_abl_$v.so 4096 2>/dev/null | sed "s/^/$v run $i: /" >> $O/ab/local.log || exit 1
  done
done
cat $O/ab/local.log
bash tools/r05_gnn_ab.sh "$@"
