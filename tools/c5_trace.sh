# C5 only: GNN-related GPU tests, then the kernel-trace stats of the C5 bench line
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests/test_gpu_gnn.py tests/test_gpu_longhorizon.py tests/test_gpu_ddp_native.py tests/test_gpu_trainer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c5_tests.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c5 -o run -- python3 $R/bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-pcie > $R/gpurun_out/prof/c5.log 2>&1
cp /tmp/prof_c5/run_kernel_stats.csv $R/gpurun_out/prof/c5_kernel_stats.csv
