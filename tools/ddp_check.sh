set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddp_native.py tests/test_gpu_trainer.py -x -v --timeout 120 --timeout-method thread > gpurun_out/ddp_tests.log 2>&1
for loop in native python; do
DDRL_FORCE_DDP=1 DDRL_DDP_LOOP=$loop timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 2 --warmup 1 --no-cpu-baseline --no-pcie --ddp-mode split > gpurun_out/ddp_bench_$loop.log 2>&1
done
