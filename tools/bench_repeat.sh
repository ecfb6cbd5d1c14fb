# default bench line, short, repeated (timing noise of the update latency); arg: repeats
set -e
mkdir -p gpurun_out
for i in $(seq 1 ${1:-3}); do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pcie > gpurun_out/rep_$i.log 2>&1
  python3 -c "import json; r=json.loads(open('gpurun_out/rep_$i.log').read().strip().splitlines()[-1]); print('run $i', round(r['value']), 'latency_us', round(r['ppo_update_ms_per_minibatch_latency']*1e3,3))"
done
