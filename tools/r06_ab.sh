#!/bin/bash
# r06 A/B timing: the default library against the in-tree variant builds named on the command line
# (tools/ablate.py build), Local and C4 update us/step at 4096 envs, three alternating rounds; the
# state digest shows bit-identity.
O=gpurun_out/r06/ab
mkdir -p $O
for i in 1 2 3; do
  for v in default "$@"; do
    lib=$(pwd)/ddrl_amd/libddrl_hip.so
    [ "$v" = default ] || lib=$(pwd)/ddrl_amd/libddrl_hip_abl_$v.so
    timeout -k 10 120 python tools/ablate.py one $lib 4096 2>/dev/null | sed "s/^/local $v run $i: /" >> $O/timing.log || exit 1
    timeout -k 10 120 python -c "import sys; sys.argv=['x']; sys.path.insert(0,'tools'); import ablate; ablate.one('$lib', 4096, 'QuantrupedMultiEnv_SharedDecentral')" 2>/dev/null | sed "s/^/c4 $v run $i: /" >> $O/timing.log || exit 1
  done
done
cat $O/timing.log
