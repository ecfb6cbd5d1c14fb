set -o pipefail
mkdir -p gpurun_out/r03abl
timeout -k 10 500 python -u tools/ablate.py run 4096 "" DDRL_ABL_NO_HEADDPP DDRL_ABL_NO_ADAM DDRL_ABL_NO_EXCHANGE DDRL_ABL_NO_DW1 DDRL_ABL_NO_DW2 DDRL_ABL_NO_L2BWD > gpurun_out/r03abl/ablate.log 2>&1
