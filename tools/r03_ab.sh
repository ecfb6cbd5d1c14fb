# usage: bash tools/r03_ab.sh tag1 tag2 ...   (libddrl_hip_abl_<tag>.so); parity on the last tag, timing of all
set -o pipefail
mkdir -p gpurun_out/ab
last=${@: -1}
DDRL_LIB=$(pwd)/ddrl_amd/libddrl_hip_abl_$last.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_longhorizon.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/tests_$last.log 2>&1; echo "tests rc=$?" >> gpurun_out/ab/tests_$last.log
for i in 1 2; do
  for v in "$@"; do
    timeout -k 10 100 python tools/ablate.py one $(pwd)/ddrl_amd/libddrl_hip_abl_$v.so 4096 2>/dev/null | sed "s/^/$v run $i: /" >> gpurun_out/ab/timing.log
  done
done
