#!/bin/bash
# r04: the tests touched by the ADVICE / target-velocity changes, a short bench, the counter list.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/c1
timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/c1/avail.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_hostenv.py -x -v --timeout 120 --timeout-method thread > gpurun_out/c1/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c1/bench.log 2>&1 || exit 1
