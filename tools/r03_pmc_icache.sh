set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r03ic
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|WAIT_INST|INST_LEVEL|SQC" $OUT/avail.txt | head -60 > $OUT/avail_ic.txt || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $OUT/p1 -o run -- python3 $R/tools/ablate.py one $R/ddrl_amd/libddrl_hip_abl_base.so 512 > $OUT/p1.log 2>&1
