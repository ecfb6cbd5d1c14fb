set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03ic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/p2 -o run -- python3 $R/tools/ablate.py one $R/ddrl_amd/libddrl_hip_abl_base.so 512 > $OUT/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES --output-format csv -d $OUT/p3 -o run -- python3 $R/tools/ablate.py one $R/ddrl_amd/libddrl_hip_abl_base.so 512 > $OUT/p3.log 2>&1
