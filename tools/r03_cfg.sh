set -o pipefail
mkdir -p gpurun_out/cfg
timeout -k 10 300 python -u bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/cfg/c4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-pcie > gpurun_out/cfg/c5.log 2>&1 &&
DDRL_STAMPS_LIB=1 timeout -k 10 200 python -u tools/diag_stamps.py 4096 > gpurun_out/cfg/stamps.log 2>&1
