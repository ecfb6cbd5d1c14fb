#!/bin/bash
# Round-1 profile recipe (run on the GPU box from the repo root):
#   kernel-trace stats of the bench, then one PMC pass per TCC counter (FETCH_SIZE and
#   WRITE_SIZE do not fit one pass), then the default bench with the CPU baseline.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/pmc_write.log 2>&1
cd $R
# the bench reports traffic from profiles/r01/pmc_update.json: refresh it from these passes
python3 tools/pmc_summary.py $OUT > $OUT/pmc_update.json
cp $OUT/pmc_update.json $R/profiles/r01/pmc_update.json
timeout -k 10 400 python3 bench.py > $OUT/bench_default.log 2>&1
