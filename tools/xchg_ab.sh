set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_bounds.py tests/test_gpu_parity.py -x -q --timeout 150 --timeout-method thread -k "bounds or update or schedule or ddp" > gpurun_out/x_tests.log 2>&1
for v in default coherent atomic; do
  if [ $v = coherent ]; then export DDRL_XCHG_COHERENT=1; else unset DDRL_XCHG_COHERENT; fi
  if [ $v = atomic ]; then export DDRL_LIB=libddrl_hip_atomic.so; else unset DDRL_LIB; fi
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/x_bench_$v.log 2>&1
  python3 -c "import json; r=json.loads(open('gpurun_out/x_bench_$v.log').read().strip().splitlines()[-1]); print('$v', round(r['value']), 'latency_us', round(r['ppo_update_ms_per_minibatch_latency']*1e3,3))"
done
