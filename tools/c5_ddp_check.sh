set -e
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 DDRL_FORCE_DDP=1
for loop in native python; do
DDRL_DDP_LOOP=$loop timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 512 --steps 1 --warmup 1 --no-pcie --ddp-mode split > gpurun_out/c5_ddp_$loop.log 2>&1
done
