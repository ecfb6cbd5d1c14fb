#!/bin/bash
# r04 evidence in one call (GPU box, repo root): the whole GPU suite, smoke(), the bench lines
# (Local default, C4, C5 one-launch and three-launch) and the GNN phase timeline.  Every step has
# its own limit; the first failure ends the script (SKIP_GNN_EXTRA=1: no three-launch line or
# timeline).  Profiles: tools/profile_r04.sh.
set -o pipefail
O=gpurun_out/all
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench_default.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_c4.log 2>&1 || exit 1
B5="--env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie"
timeout -k 10 300 python3 bench.py $B5 > $O/bench_c5.log 2>&1 || exit 1
[ -n "$SKIP_GNN_EXTRA" ] && exit 0
DDRL_GNN_TAIL=0 timeout -k 10 300 python3 bench.py $B5 > $O/bench_c5_3launch.log 2>&1 || exit 1
timeout -k 10 240 python -u tools/diag_gnn_stamps.py 2048 mpnn > $O/stamps_gnn_mpnn.log 2>&1 || exit 1
