#!/bin/bash
# GPU loop for data-parallel step changes: the DDP / update parity tests, then the DDP profile.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddp_native.py tests/test_gpu_trainer.py tests/test_gpu_parity.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/ddp_iter_tests.log 2>&1
bash tools/profile_ddp.sh
