set -e
bash tools/bench_repeat.sh 2
export DDRL_LIB=libddrl_hip_old.so
bash tools/bench_repeat.sh 2
