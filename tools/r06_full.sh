#!/bin/bash
# Round-6 full GPU pass (run on the GPU box from the repo root): the whole GPU suite, smoke(),
# the peer-mode timing and the default bench line.  Each GPU step has its own time limit and the
# first failure ends the run.
set -o pipefail
out=gpurun_out/r06
mkdir -p $out
timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 600 --timeout-method thread tests/ > $out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
tail -3 $out/smoke.log
timeout -k 10 400 python3 bench.py > $out/bench_default.log 2>&1 || exit $?
tail -c 1200 $out/bench_default.log
