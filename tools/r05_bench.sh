#!/bin/bash
# r05 bench lines (GPU box, repo root): the default bench as the driver runs it, C4, C5 (one
# launch, and three launches), the data-parallel learner at one rank (C4, C5), and the smoke test.
set -o pipefail
O=gpurun_out/r05/bench
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.log 2>&1 || exit 1
tail -c 400 $O/bench_default.log; echo
timeout -k 10 400 python3 bench.py --env QuantrupedMultiEnv_SharedDecentral --steps 2 --warmup 1 > $O/bench_c4.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || exit 1
DDRL_GNN_TAIL=0 timeout -k 10 400 python3 bench.py --env QuantrupedMultiEnv_DecentralShared_Graph --envs 2048 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_c5_3launch.log 2>&1 || exit 1
for e in "QuantrupedMultiEnv_SharedDecentral 4096" "QuantrupedMultiEnv_DecentralShared_Graph 2048"; do
  set -- $e
  DDRL_FORCE_DDP=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --env $1 --envs $2 --steps 1 --warmup 1 --no-cpu-baseline --no-pcie > $O/bench_${1}_ddp1.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/r05/bench/bench_*.log")):
    r = json.loads([l for l in open(f).read().splitlines() if l.startswith("{")][-1])
    cb = r.get("cpu_baseline", {})
    print(f.split("/")[-1], round(r["value"]), "env-steps/s", round(r["ppo_update_ms_per_minibatch_latency"] * 1e3, 3), "us/step",
          "frac", round(r["roofline"]["frac"], 4), "cpu", round(cb.get("value", 0), 1))
PY
tail -2 $O/smoke.log
