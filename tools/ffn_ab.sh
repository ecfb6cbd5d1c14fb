# fcnet update kernel A/B: default bench line (short) per variant library, alternating, and
# the parity tests on the variant; args: variant names (libddrl_hip_<v>.so)
set -e
mkdir -p gpurun_out
for v in "$@"; do
  DDRL_LIB=libddrl_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests_$v.log 2>&1
done
for i in 1 2; do
  for v in prod "$@"; do
    lib=libddrl_hip.so; [ "$v" = prod ] || lib=libddrl_hip_$v.so
    DDRL_LIB=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/ab_$v.log 2>&1
    python3 -c "import json; r=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]); print('$v run $i', round(r['value']), 'latency_us', round(r['ppo_update_ms_per_minibatch_latency']*1e3,3))"
  done
done
