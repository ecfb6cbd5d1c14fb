#!/bin/bash
# Round-5 GPU check (run on the GPU box from the repo root): the placement guard, the LSB-exchange
# bound and the full-size shared-policy tests, then the C5 bench line with its CPU baseline and
# a short default bench.  Every GPU step has its own time limit; the first failure ends the run.
set -o pipefail
mkdir -p gpurun_out/r05
out=gpurun_out/r05
timeout -k 10 420 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_gnn_rollback.py tests/test_gpu_lsb.py tests/test_gpu_gnn.py > $out/tests_new.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 $out/tests_new.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v -s --timeout 580 --timeout-method thread \
  tests/test_gpu_fullsize_shared.py > $out/tests_fullsize_shared.log 2>&1
rc=$?; echo "fullsize shared rc=$rc"; tail -5 $out/tests_fullsize_shared.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 2 --warmup 1 \
  --no-pcie > $out/bench_c5.log 2>&1 || exit $?
tail -c 1500 $out/bench_c5.log
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-pcie --no-cpu-baseline > $out/bench_default.log 2>&1 || exit $?
tail -c 600 $out/bench_default.log
