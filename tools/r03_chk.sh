set -o pipefail
mkdir -p gpurun_out/chk
DDRL_LIB=libddrl_hip_cand.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hostenv.py tests/test_gpu_fullsize.py tests/test_gpu_gnn.py tests/test_gpu_checkpoint.py -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/tests.log 2>&1
echo "rc=$?" >> gpurun_out/chk/tests.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/chk/bench_pk.log 2>&1
DDRL_LIB=libddrl_hip_cand.so timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/chk/bench_cand.log 2>&1
bash tools/r03_time.sh pk fn
