# A/B of the exchange protocols (GPU box, repo root): the production L2 protocol vs the
# relaxed agent-scope atomic build (python -m ddrl_amd.build --atomic), short default benches.
set -e
bash tools/bench_repeat.sh 2
export DDRL_LIB=libddrl_hip_atomic.so
bash tools/bench_repeat.sh 2
