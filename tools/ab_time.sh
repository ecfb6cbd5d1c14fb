# usage: bash tools/ab_time.sh tag1 tag2 ...  : us/step of libddrl_hip_abl_<tag>.so at 4096 envs, 2 rounds
mkdir -p gpurun_out/ab
for i in 1 2; do
  for v in "$@"; do
    timeout -k 10 100 python tools/ablate.py one $(pwd)/ddrl_amd/libddrl_hip_abl_$v.so 4096 2>/dev/null | sed "s/^/$v run $i: /" >> gpurun_out/ab/timing.log
  done
done
