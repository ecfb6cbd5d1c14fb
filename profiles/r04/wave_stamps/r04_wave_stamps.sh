#!/bin/bash
# r04: per-wave phase stamps of the fused update (Local, 4096 envs): the diagnostic build
# stamped on lane 0 of wave 0 (libddrl_hip_stamps.so) and of waves 1-3 (libddrl_hip_stw<tid>.so,
# -DDDRL_STAMP_TID=<tid>), each prebuilt here.
set -o pipefail
mkdir -p gpurun_out/stw
for l in libddrl_hip_stamps.so libddrl_hip_stw64.so libddrl_hip_stw128.so libddrl_hip_stw192.so; do
  DDRL_STAMPS_LIB=$l timeout -k 10 200 python tools/diag_stamps.py 4096 > gpurun_out/stw/$l.log 2>&1 || exit 1
done
