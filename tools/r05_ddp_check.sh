set -o pipefail
O=gpurun_out/r05/ddp
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_ddp_native.py tests/test_gpu_rollback.py tests/test_gpu_bounds.py tests/test_gpu_gnn_rollback.py > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for e in "QuantrupedMultiEnv_SharedDecentral 4096" "QuantrupedMultiEnv_DecentralShared_Graph 2048"; do
  set -- $e
  DDRL_FORCE_DDP=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --env $1 --envs $2 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_${1}_ddp1.log 2>&1 || exit 1
  grep -o '"ppo_update_ms_per_minibatch_latency": [0-9.]*' $O/bench_${1}_ddp1.log
done
