set -o pipefail
mkdir -p gpurun_out/ab
bash tools/r03_time.sh "$@"
DDRL_STAMPS_LIB=1 timeout -k 10 200 python -u tools/diag_stamps.py 4096 > gpurun_out/ab/stamps.log 2>&1
