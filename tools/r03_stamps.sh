set -o pipefail
mkdir -p gpurun_out/st
for v in libddrl_hip_stamps.so libddrl_hip_stamps_np.so; do
DDRL_STAMPS_LIB=$v timeout -k 10 200 python -u tools/diag_stamps.py 4096 > gpurun_out/st/$v.log 2>&1 || exit 1
done
