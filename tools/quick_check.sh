#!/bin/bash
# Quick GPU loop for update-kernel changes (run on the GPU box from the repo root):
# the update parity tests, then a short default bench (no CPU baseline / PCIe leg).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cup.py -x -q --timeout 120 \
  --timeout-method thread -k "update or schedule or ddp or cup" > gpurun_out/quick_tests.log 2>&1
timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/quick_bench.log 2>&1
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/quick_bench.log").read().strip().splitlines()[-1])
print("value", round(r["value"]), "latency_us", round(r["ppo_update_ms_per_minibatch_latency"] * 1e3, 3))
PY
