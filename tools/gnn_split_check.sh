# GNN forward split: GNN-related GPU tests on the production library, the GNN tests again on
# the atomic-exchange build, then the C5 bench line on both
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_longhorizon.py tests/test_gpu_ddp_native.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gs_tests.log 2>&1
DDRL_LIB=libddrl_hip_atomic.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gnn.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gs_tests_atomic.log 2>&1
for v in "" atomic; do
  lib=ddrl_amd/libddrl_hip${v:+_$v}.so
  DDRL_LIB=$PWD/$lib timeout -k 10 200 python bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/gs_${v:-prod}.log 2>&1
  python3 -c "import json; r=json.loads(open('gpurun_out/gs_${v:-prod}.log').read().strip().splitlines()[-1]); print('${v:-prod}', round(r['value']), 'latency_us', round(r['ppo_update_ms_per_minibatch_latency']*1e3,3))"
done
