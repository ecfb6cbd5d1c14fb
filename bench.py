"""DDRL rollout + multi-agent PPO update on MI355X: env-steps/s at 4096 envs x 4 leg agents.

One bench step = one PPO training iteration of the reference's exp-1 trainer on the
QuantrupedMultiEnv_Local configuration (4 independent per-leg fcnet 2x64 policies, d = 35):
  rollout of rollout_fragment_length = 200 vector env-steps over this rank's envs
    (env-side MeanStdFilter + routing, fused forward of the 4 policies + DiagGaussian
     sampling, per-leg rewards; synthetic QuAntruped data resident in HBM),
  bootstrap V(s_T), GAE + advantage standardization,
  SampleBatch shuffle + per-epoch minibatch permutations,
  PPO update: num_sgd_iter = 10 epochs x (R / 128) minibatches per policy, all 4 policies
    concurrently (fused persistent kernel: forward, PPOLoss, backward, clip, Adam),
  KL-coefficient update from the last epoch's mean KL (host).
Multi-GPU: 4096 envs are sharded over the ranks (C3: independent policies, no collective);
each rank is an independent learner on its shard ("replicas"), value = all ranks' env-steps
divided by the slowest rank's time.  Shared-policy envs (--env QuantrupedMultiEnv_SharedDecentral,
..._DecentralShared_Graph) default to gather mode at N > 1: every rank rolls out its shard, one
all-gather of the records per iteration, and every rank runs the same fused update over the union
batch -- the single-GPU algorithm exactly, the fastest exact mode.
--shared-mode ddp trains data-parallel instead (RCCL all-reduce of the gradient every SGD step):
the library's RCCL loop (ddrl_ppo_update_ddp) by default, DDRL_DDP_LOOP=python for the Python
loop, --ddp-mode split | local (ddrl_amd/ddp.py).  DDRL_FORCE_DDP=1 runs that learner at one rank
(under torchrun) and DDRL_DIST_BACKEND=gloo rehearses N ranks on one GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 4096] [--env NAME] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

def metric_name(envs):
    """BASELINE.json's metric, with the env count of this run (4096 = the metric's config)."""
    return f"env-steps/sec at {envs} envs × 4 leg agents; PPO update ms/minibatch"
PEAK_FP32_TFLOPS = 157.3   # MI355X dense FP32 (MFMA f32 = vector rate), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0
PMC_SUMMARIES = [os.path.join(ROOT, "profiles", r, "pmc_summary.json") for r in ("r06", "r05", "r04", "r03")]
PMC_WORKLOAD = {"QuantrupedMultiEnv_Local": "local", "QuantrupedMultiEnv_SharedDecentral": "c4",
                "QuantrupedMultiEnv_DecentralShared_Graph": "c5"}


def pmc_key(env, gnn_tail=True):
    """Workload key of the committed PMC passes; the three-launch GNN step has its own pass."""
    k = PMC_WORKLOAD.get(env, "")
    return k + "_3launch" if k == "c5" and not gnn_tail else k


def pmc_summary(key=None):
    """The newest committed rocprofv3 PMC summary (tools/pmc_summary.py) that holds `key` (any,
    when None), and its path."""
    for path in PMC_SUMMARIES:
        try:
            with open(path) as f:
                s = json.load(f)
        except OSError:
            continue
        if key is None or key in s.get("workloads", {}):
            return s, os.path.relpath(path, ROOT)
    return None, None


def pmc_workload(key):
    s, path = pmc_summary(key)
    return (s or {}).get("workloads", {}).get(key), path


def pmc_traffic(key, policy_steps):
    """HBM bytes of the update (all its launches) from the committed rocprofv3 PMC passes
    (FETCH_SIZE x 2 per the gfx950 correction + WRITE_SIZE; tools/profile_r06.sh): the
    workload's bytes per (policy, minibatch) step times this update's steps -- the kernels'
    traffic is per step.  The counters cannot be read live from inside the timed run; None
    for a workload without a committed pass."""
    w, _ = pmc_workload(key)
    return w["hbm_bytes_per_step"] * policy_steps if w else None


def pmc_ns_per_step(key, P):
    """Duration per sequential minibatch step of the dominant kernel in the committed PMC pass
    (its --kernel-trace duration over the pass's steps; P policies run side by side), or None."""
    w, _ = pmc_workload(key)
    m = (w or {}).get("mfma") or {}
    if not m.get("duration_ns") or not w.get("steps"):
        return None
    return m["duration_ns"] / (w["steps"] / P)


# the configurations tools/profile_r06.sh traces (bench defaults): envs per workload key.  The
# three-launch C5 step is left out: under the tracer its 38,400 short dispatches per epoch carry
# the tracer's per-dispatch cost (its trace sums to 21.7 us per step against 18.9 us untraced)
PROFILED_ENVS = {"local": 4096, "c4": 4096, "c5": 2048}


def trace_ns_per_step(key, steps_per_dispatch):
    """The dominant kernel's time per sequential step in the kernel-trace pass (no counters) that
    the same recipe took beside the PMC passes: prof/<key>_kernel_stats.csv next to the summary.
    The PMC passes themselves run slower where a step is a dispatch of its own (C5: the counters
    are read around every one of 12,800 dispatches, +15 %), so the trace pass is the one compared
    with this run."""
    import csv
    _, path = pmc_summary(key)
    if path is None:
        return None
    d = os.path.join(ROOT, os.path.dirname(path))
    for f in (os.path.join(d, "prof", f"{key}_kernel_stats.csv"), os.path.join(d, f"{key}_kernel_stats.csv")):
        if os.path.exists(f):
            with open(f) as fh:
                rows = list(csv.DictReader(fh))
            ns = float(rows[0]["AverageNs"])
            if key == "c5_3launch":   # the step's other two launches
                ns += sum(float(r["AverageNs"]) for r in rows if r["Name"].startswith(("k_gnn_reduce", "k_gnn_adam")))
            return ns / steps_per_dispatch
    return None


def pmc_mfma(key):
    """MFMA-busy and effective clock of the workload's dominant update kernel from the committed
    counter pass (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE with --kernel-trace; see
    tools/pmc_summary.py for the arithmetic), or {} without one."""
    w, path = pmc_workload(key)
    m = (w or {}).get("mfma")
    if not m:
        return {}
    return {"mfma_busy_frac": m.get("mfma_busy_frac_of_active_simds"), "clock_ghz": m.get("clock_ghz"),
            "mfma_busy_frac_chip": m.get("mfma_busy_frac_chip"), "mfma_source": f"{path} ({m.get('kernel')})"}


def parallel_mode(shared_mode, n_policies, world, force_ddp=False):
    """How the ranks train: "single" (one process), "replicas" (independent learners on env
    shards), "gather" (one record all-gather per iteration, the same fused
    update over the union batch on every rank: the single-GPU algorithm exactly) or "ddp" (the
    data-parallel learner, gradient all-reduce every SGD step; shared-policy envs only).
    shared_mode "auto" picks gather for a shared policy and replicas otherwise; DDRL_FORCE_DDP
    (force_ddp) names the data-parallel learner, at one rank too."""
    if world <= 1 and not force_ddp:
        return "single"
    mode = shared_mode
    if mode == "auto":
        mode = "ddp" if force_ddp else ("gather" if n_policies == 1 else "replicas")
    if mode == "ddp" and n_policies != 1:
        return "replicas"
    return mode


def ffn_flops_per_row(d, A, H=64):
    """Algorithmic FLOPs of one minibatch row through the fused update step:
    forward (policy + value) + input-gradient backward of layers 2/head + weight gradients."""
    fwd = d * H + H * H + H * 2 * A + d * H + H * H + H * 1
    dx = (H * H + H * 2 * A) + (H * H + H * 1)
    return 2 * (2 * fwd + dx)


def ffn_fwd_flops_per_row(d, A, H=64):
    return 2 * (d * H + H * H + H * 2 * A + d * H + H * H + H)


def gnn_flops_per_row(A, H=64, F=19):
    """GraphNet actor + critic on one training row (a graph of 4 nodes): per net and node
    the hypernetwork (4 x 1216), f W_n (19 x 64), message and node layers (64 x 64 each),
    the selected node's head; backward = 2 x forward (input and weight gradients, the
    hypernetwork recomputed counts once more)."""
    fwd_net = lambda O: 2 * (4 * (4 * F * H + F * H + 2 * H * H) + H * O)
    fwd = fwd_net(2 * A) + fwd_net(1)
    return 3 * fwd + 2 * 4 * 4 * F * H * 2


def _cpu_model(O, cfg, p):
    """The oracle's model of policy p: (kind, params, shapes), Glorot-initialized from a seed
    fixed per policy (the same in every worker of the parallel baseline)."""
    rng, A = np.random.default_rng(1000 + p), cfg.act_dim
    if cfg.model_kind == 1:   # "gnn" (DecentralShared_Graph): one shared GraphNet leg policy
        return "gnn", O.gnn_init(rng, 2 * A), O.gnn_param_shapes(2 * A)
    return "ffn", O.ffn_init(rng, cfg.obs_dim[p], 2 * A), O.ffn_param_shapes(cfg.obs_dim[p], 2 * A)


def _cpu_rollout(O, cfg, inst, n_envs, T, rng):
    """The oracle's rollout of one fragment over n_envs envs with its own env-side MeanStdFilter
    (as every RLlib rollout worker process has): per step filter + routing, each policy's
    forward over its rows (row c = env * k + slot for the policy's k agents), DiagGaussian
    sampling, per-leg rewards; then the bootstrap and GAE per policy.  Returns the unstandardized
    train batch of every policy."""
    P, A = cfg.n_policies, cfg.act_dim
    agents = list(inst.agent_names)
    slots = [[a for j, a in enumerate(agents) if cfg.agent_policy[j] == p] for p in range(P)]
    models = [_cpu_model(O, cfg, p) for p in range(P)]
    obs = rng.normal(size=(T + 1, n_envs, cfg.obs_full_dim)).astype(np.float32)
    eps = rng.normal(size=(T, n_envs, cfg.n_agents, A)).astype(np.float32)
    fw = rng.normal(size=(T, n_envs)).astype(np.float32)
    cfrc = rng.normal(size=(T, n_envs, 14, 6)).astype(np.float32)
    rs = O.RunningStat((cfg.obs_full_dim,))
    node_tables = [inst.obs_indices[a] for a in agents]

    def forward(p, t_obs, z):
        kind, params, _ = models[p]
        if kind == "gnn":   # X [4][23] per env, one training row per node (c = env * 4 + node)
            X = np.stack([O.graph_observation(t_obs[e].astype(np.float64), z[e], node_tables)
                          for e in range(n_envs)]).astype(np.float32)
            x, node = np.repeat(X, 4, axis=0), np.tile(np.arange(4), n_envs)
            logits, value, _ = O.gnn_forward(params, x, node)
            return (x, node), logits, value
        x = np.stack([z[:, inst.obs_indices[a]] for a in slots[p]], 1).reshape(-1, cfg.obs_dim[p]).astype(np.float32)
        logits, value, _ = O.ffn_forward(params, x)
        return (x, None), logits, value

    rec = [dict(obs=[], node=[], act=[], logits=[], logp=[], vf=[], rew=[]) for _ in range(P)]
    tables = {a: inst.contact_force_indices[a] for a in agents}
    z = O.mean_std_filter(obs[0], rs, True, 10.0)
    for t in range(T):
        actions = np.zeros((n_envs, 8))
        for p in range(P):
            (x, node), logits, value = forward(p, obs[t], z)
            ep = eps[t][:, [agents.index(a) for a in slots[p]]].reshape(-1, A)
            act = O.dg_sample(logits, ep)
            for k, v in (("obs", x), ("node", node), ("act", act), ("logits", logits),
                         ("logp", O.dg_logp(logits, act)), ("vf", value)):
                rec[p][k].append(v)
            for s, a in enumerate(slots[p]):
                actions[:, inst.action_indices[a]] = np.clip(act.reshape(n_envs, len(slots[p]), A)[:, s], -1, 1)
        rw = [O.per_leg_reward(float(fw[t, e]), cfrc[t, e], {a: actions[e, inst.action_indices[a]] for a in agents},
                               tables, 0.5, 0.05) for e in range(n_envs)]
        for p in range(P):
            rec[p]["rew"].append(np.array([[rw[e][a] for a in slots[p]] for e in range(n_envs)],
                                          np.float32).reshape(-1))
        z = O.mean_std_filter(obs[t + 1], rs, True, 10.0)
    out = []
    for p in range(P):
        r = rec[p]
        last_v = forward(p, obs[T], z)[2]
        vf, rew = np.stack(r["vf"]), np.stack(r["rew"])
        adv, vt = O.gae_fragment(rew, vf, np.zeros(rew.shape, bool), last_v)
        b = dict(actions=np.concatenate(r["act"]), logits=np.concatenate(r["logits"]),
                 logp=np.concatenate(r["logp"]), vf_preds=vf.reshape(-1), adv=adv.reshape(-1), vt=vt.reshape(-1))
        if models[p][0] == "gnn":
            b.update(X=np.concatenate(r["obs"]), node_idx=np.concatenate(r["node"]))
        else:
            b.update(obs=np.concatenate(r["obs"]))
        out.append(b)
    return out


def _cpu_update(O, cfg, p, batch, rng):
    """One policy's minibatch SGD chain over its batch (10 epochs; sequential by construction:
    every step needs the previous step's weights)."""
    kind, params, shapes = _cpu_model(O, cfg, p)
    adv, _, _ = O.standardize(batch["adv"])
    sh, pe = O.sgd_schedule(rng, len(adv), 128, cfg.num_sgd_iter)
    adam = O.Adam(sum(int(np.prod(s)) for _, s in shapes))
    O.ppo_update(kind, params, shapes, adam, dict(batch, adv=adv), sh, pe, np.float32(0.2), {})


def cpu_sample_envs(env, cpu_envs):
    """Envs of the bounded CPU sample (about 10-30 s of CPU work on the GPU box): cpu_envs for
    the fcnet envs, cpu_envs / 16 for the GraphNet, whose numpy step costs ~20x the fcnet's."""
    from ddrl_amd.spec import make_cfg
    cfg, _ = make_cfg(env, 1, 1)
    return max(4, cpu_envs // 16) if cfg.model_kind == 1 else cpu_envs


def cpu_baseline(env, n_envs=128, T=200, seed=0, threads=1):
    """The numpy oracle on a bounded sample of the same workload (same env and model, same PPO
    schedule, fewer envs), BLAS limited to `threads` threads.  Returns env-steps/s."""
    from threadpoolctl import threadpool_limits
    from oracle import ddrl_oracle as O
    from ddrl_amd.spec import make_cfg
    cfg, inst = make_cfg(env, n_envs, T)
    rng = np.random.default_rng(seed)
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        batches = _cpu_rollout(O, cfg, inst, n_envs, T, rng)
        for p in range(cfg.n_policies):
            _cpu_update(O, cfg, p, batches[p], rng)
        dt = time.perf_counter() - t0
    R = len(batches[0]["adv"])
    return T * n_envs / dt, dt, f"{env}: {n_envs} envs x T={T} (full iteration: rollout, GAE, " \
                                f"{cfg.num_sgd_iter} x {R // 128} minibatches x {cfg.n_policies} " \
                                f"{'GraphNet' if cfg.model_kind == 1 else 'fcnet'} polic" \
                                f"{'y' if cfg.n_policies == 1 else 'ies'})"


def _cpu_rollout_chunk(a):
    """One rollout worker of the parallel CPU baseline: its own envs and its own env-side
    MeanStdFilter, T steps, then GAE per policy."""
    env, n_envs, T, seed = a
    from threadpoolctl import threadpool_limits
    from oracle import ddrl_oracle as O
    from ddrl_amd.spec import make_cfg
    with threadpool_limits(limits=1):
        cfg, inst = make_cfg(env, n_envs, T)
        return _cpu_rollout(O, cfg, inst, n_envs, T, np.random.default_rng(seed))


def _cpu_update_policy(a):
    """One policy's minibatch SGD chain over the union batch."""
    env, p, batch, seed = a
    from threadpoolctl import threadpool_limits
    from oracle import ddrl_oracle as O
    from ddrl_amd.spec import make_cfg
    with threadpool_limits(limits=1):
        cfg, _ = make_cfg(env, 1, 1)
        _cpu_update(O, cfg, p, batch, np.random.default_rng(seed))
    return p


def cpu_baseline_parallel(env, n_envs=512, T=200, workers=16, seed=0):
    """The iteration of cpu_baseline on `workers` host processes, parallel where the algorithm
    is: the rollout over env chunks (one env-side filter per worker, like RLlib's rollout
    workers), the PPO update over the independent policies (each policy's minibatch chain is
    sequential; the 4 leg policies train side by side).  The pool is warmed before timing.
    Run it in a process that has not initialised the GPU (bench.py starts a child for it)."""
    import multiprocessing as mp
    from ddrl_amd.spec import make_cfg
    cfg, _ = make_cfg(env, n_envs, T)
    P = cfg.n_policies
    chunks = [c for c in (n_envs // workers + (1 if w < n_envs % workers else 0) for w in range(workers)) if c]
    with mp.get_context("fork").Pool(len(chunks)) as pool:
        pool.map(_cpu_rollout_chunk, [(env, 2, 2, 99)] * len(chunks))   # warm: imports in every worker
        t0 = time.perf_counter()
        parts = pool.map(_cpu_rollout_chunk, [(env, c, T, seed + 17 * w) for w, c in enumerate(chunks)])
        batches = [{k: np.concatenate([pt[p][k] for pt in parts]) for k in parts[0][p]} for p in range(P)]
        pool.map(_cpu_update_policy, [(env, p, batches[p], seed + 5 + p) for p in range(P)])
        dt = time.perf_counter() - t0
    return T * n_envs / dt, dt, len(chunks)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--envs", type=int, default=4096, help="total envs over all ranks")
    ap.add_argument("--env", default="QuantrupedMultiEnv_Local")
    ap.add_argument("--frag", type=int, default=200)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) iteration")
    ap.add_argument("--cpu-envs", type=int, default=512)
    ap.add_argument("--sgd-iter", type=int, default=None,
                    help="profiling aid: num_sgd_iter of the run (default: the config's 10 epochs)")
    ap.add_argument("--ddp-mode", default="split", choices=["split", "local"],
                    help="shared-policy envs on N>1 GPUs: per-rank rows per SGD step (see ddrl_amd/ddp.py); "
                         "split (default) = the reference's 128-row minibatch SGD, local = 128 rows per rank")
    ap.add_argument("--shared-mode", default="auto", choices=["auto", "ddp", "gather"],
                    help="N>1 GPUs: 'gather' (records all-gathered once per iteration, every rank runs the same "
                         "fused update over the union batch: the single-GPU algorithm exactly, no per-step "
                         "collective), 'ddp' (shared-policy envs: RCCL all-reduce of the gradient every SGD "
                         "step) or 'auto' (default): gather for shared-policy envs -- the fastest exact mode "
                         "(DESIGN.md section 5) -- and replicas for independent-policy envs")
    args = ap.parse_args()

    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DDRL_DIST_BACKEND=gloo rehearses the multi-rank path on one GPU (ranks share device 0,
    # the end-of-run reductions go over gloo on the host); the default is RCCL ("nccl")
    backend = os.environ.get("DDRL_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    # DDRL_FORCE_DDP=1 runs the data-parallel learner even at one rank (torchrun, world 1):
    # the RCCL path of the shared-policy configurations exercised on a one-GPU box
    force_ddp = os.environ.get("DDRL_FORCE_DDP") == "1"
    dist = None
    if world > 1 or force_ddp:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from ddrl_amd import native as N
    from ddrl_amd.build import build
    from ddrl_amd.spec import make_cfg
    from ddrl_amd.synthetic import SyntheticRollout
    if rank == 0 and not os.path.exists(N.LIB_PATH):
        build()
    if dist is not None:
        dist.barrier()

    n_local = args.envs // world + (1 if rank < args.envs % world else 0)
    T = args.frag
    run_config = {"num_sgd_iter": args.sgd_iter} if args.sgd_iter else None
    cfg, inst = make_cfg(args.env, n_local, T, run_config)
    stream = torch.cuda.current_stream()
    ctx = N.Context(cfg, local, stream.cuda_stream)
    P, A = cfg.n_policies, cfg.act_dim
    gnn = cfg.model_kind == N.MODEL_GNN
    # shared-policy envs on several GPUs train data-parallel (identical weights on every
    # rank); independent-policy envs are replicas (own weights per rank)
    mode = parallel_mode(args.shared_mode, P, world, force_ddp)
    ddp, gather = mode == "ddp", mode == "gather"
    if gather and args.envs % world:
        raise SystemExit("--shared-mode gather needs --envs divisible by the number of ranks")
    rng = np.random.default_rng(1234 if (ddp or gather) else 1234 + rank)
    from ddrl_amd.trainer import glorot_ffn_flat
    from ddrl_amd.models import glorot_gnn_flat
    for p in range(P):
        ctx.params_set(p, glorot_gnn_flat(rng, A) if gnn else glorot_ffn_flat(rng, cfg.obs_dim[p], A))
    syn = SyntheticRollout(n_local, T, cfg.obs_full_dim, cfg.n_agents, A, f"cuda:{local}", seed=rank)
    kl = [0.2] * P
    R = [T * ctx.layout[p]["C"] for p in range(P)]
    nb = [max(1, r // 128) for r in R]
    E = cfg.num_sgd_iter
    gen = torch.Generator(device=f"cuda:{local}")
    gen.manual_seed(99 if gather else 99 + rank)   # gather: the same schedule on every rank
    uctx = None
    if gather:
        # the learner context: the union batch of all ranks (rank-major), same weights everywhere
        ucfg, _ = make_cfg(args.env, n_local * world, T, run_config)
        uctx = N.Context(ucfg, local, stream.cuda_stream)
        for p in range(P):
            uctx.params_set(p, ctx.params_get(p))
        R = [T * uctx.layout[p]["C"] for p in range(P)]
        nb = [max(1, r // 128) for r in R]
        from ddrl_amd.ddp import Comm, gather_records, sync_standardize, standardize_constants
        comm = Comm(f"cuda:{local}" if backend == "nccl" else "cpu") if dist is not None else None
    ev_upd = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    upd_ms = []
    if ddp:
        from ddrl_amd.ddp import (Comm, DataParallelLearner, HipBackend, NativeDataParallelLearner,
                                  native_comm_init, sync_standardize)
        comm = Comm(f"cuda:{local}" if backend == "nccl" else "cpu")
        if backend == "nccl" and os.environ.get("DDRL_DDP_LOOP", "native") == "native":
            # the minibatch loop inside the library on its own RCCL communicator
            native_comm_init(ctx, comm)
            learner = NativeDataParallelLearner(ctx, comm, 0, 128, args.ddp_mode)
        else:
            learner = DataParallelLearner(HipBackend(ctx), comm, 0, 128, args.ddp_mode)
        grad = torch.zeros(ctx.n_params[0], dtype=torch.float32, device=f"cuda:{local}")
        sched_rng = np.random.default_rng(77 + rank)

    ctx.observe(syn.obs[0])

    henv = None
    host_threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))

    def rollout_host_env(groups=2):
        """The rollout with the envs stepped on the host (f1): the C++ thread pool steps the
        QuAntruped stand-in into pinned buffers, pipelined over env groups so that one
        group's host step overlaps the device's reward / observe / act of the other and the
        PCIe transfers (ddrl_rollout_hostenv).  The first call resets the envs."""
        nonlocal henv
        first = henv is None
        if first:
            henv = N.HostEnv(n_local, cfg.obs_full_dim, host_threads, seed=1000 + rank)
        ctx.rollout_hostenv(henv, syn.eps, groups=groups, reset=first)

    def iteration(record, host_io=False):
        done = syn.dones_for_fragment()
        if host_io:
            rollout_host_env()
        else:
            # T x (act, reward, observe) + bootstrap in one C-ABI call (device-resident env data)
            ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, done, syn.actions)
        ctx.gae()
        if ddp:
            # the env-side MeanStdFilter stays rank-local (a per-process singleton in the
            # reference, simulation_envs/observation_filter.py:3-12: never synchronized)
            ctx.adv_norm_set(0, *sync_standardize(comm, ctx.adv_sums_get(0)))
            sh, pe = learner.schedule(sched_rng, R[0], E)
            sh_dev = torch.from_numpy(sh).to(stream.device)
            ev_upd[0].record(stream)
            mkl = learner.learn(sh_dev, pe, kl[0], grad)
            ev_upd[1].record(stream)
            kl[0] = kl[0] * 1.5 if mkl > 2 * 0.01 else (kl[0] * 0.5 if mkl < 0.5 * 0.01 else kl[0])
            if record:
                torch.cuda.synchronize()
                upd_ms.append(ev_upd[0].elapsed_time(ev_upd[1]))
                steps_done.append(pe.size)
            return
        lctx = ctx
        if gather:
            lctx = uctx
            for p in range(P):
                sums = ctx.adv_sums_get(p)
                uctx.adv_norm_set(p, *(sync_standardize(comm, sums) if comm else standardize_constants(sums)))
                gather_records(comm, ctx.records_tensor(p), uctx.records_tensor(p))
        # SampleBatch.shuffle + per-epoch minibatch permutations of every policy: one batched
        # argsort of fp64 uniforms each (policies of one env have equal batch sizes)
        if len(set(R)) == 1:
            dev = stream.device
            sh_all = torch.rand((P, R[0]), device=dev, generator=gen, dtype=torch.float64).argsort(dim=1)
            pe_all = torch.rand((P, E, nb[0]), device=dev, generator=gen, dtype=torch.float64).argsort(dim=2)
            sh_all, pe_all = sh_all.to(torch.int32), pe_all.to(torch.int32)
            shuffles = [sh_all[p] for p in range(P)]
            perms = [pe_all[p] for p in range(P)]
        else:
            shuffles = [torch.randperm(R[p], device=stream.device, generator=gen, dtype=torch.int32) for p in range(P)]
            perms = [torch.stack([torch.randperm(nb[p], device=stream.device, generator=gen, dtype=torch.int32)
                                  for _ in range(E)]).contiguous() for p in range(P)]
        ev_upd[0].record(stream)
        lctx.ppo_update((1 << P) - 1, shuffles, perms, kl)
        try:
            lctx.synchronize()
        except N.DdrlError as e:
            # a failed update restored its state; a context that has switched protocol (the
            # atomic exchange after a broken placement, the three-launch GNN step after an
            # abandoned wait -- e.g. a GPU shared with other processes' grids) asks for the
            # update again, which is the same update on the same state
            if "call the update again" not in str(e):
                raise
            print(f"bench: rank {rank}: {e} -- running the update again", file=sys.stderr, flush=True)
            lctx.ppo_update((1 << P) - 1, shuffles, perms, kl)
        ev_upd[1].record(stream)
        if gather:   # the next rollout uses the updated weights
            for p in range(P):
                ctx.params_set(p, uctx.params_get(p))
        # RLlib: update_kl with the last epoch's mean KL of every policy
        for p in range(P):
            st = lctx.ppo_stats(p, nb[p], first=(E - 1) * nb[p])   # the last epoch's rows
            mkl = float(np.mean(st[:, 3]))
            kl[p] = kl[p] * 1.5 if mkl > 2 * 0.01 else (kl[p] * 0.5 if mkl < 0.5 * 0.01 else kl[p])
        if record:
            upd_ms.append(ev_upd[0].elapsed_time(ev_upd[1]))
            steps_done.append(E * nb[0])

    steps_done = []
    for _ in range(args.warmup):
        iteration(False)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        iteration(True)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t_max = elapsed
    env_steps = T * n_local * args.steps
    if dist is not None:
        red_dev = "cuda" if backend == "nccl" else "cpu"
        tt = torch.tensor([elapsed], device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_max = float(tt.item())
        es = torch.tensor([env_steps], device=red_dev, dtype=torch.float64)
        dist.all_reduce(es)
        env_steps = int(es.item())

    pcie = None
    if world == 1 and not args.no_pcie and not ddp:
        # as many iterations again with the envs on the host (not part of value): pipelined host env
        # plane rollout + GAE + the same update
        torch.cuda.synchronize()
        rollout_host_env()            # warm-up: resets the envs, first pinned transfers
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):   # the same number of iterations as the timed region
            iteration(False, host_io=True)
        torch.cuda.synchronize()
        it_s = (time.perf_counter() - t1) / args.steps
        ro = {}
        for groups in (1, 2):
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rollout_host_env(groups)
            torch.cuda.synchronize()
            ro[groups] = time.perf_counter() - t2
        t3 = time.perf_counter()
        for _ in range(20):
            henv.step()
        step_s = (time.perf_counter() - t3) / 20
        per_step_bytes = 4 * n_local * (cfg.obs_full_dim + 8 + 1 + 14 * 6) + n_local
        pcie = {"value": T * n_local / it_s, "unit": "env-steps/s", "iteration_ms": it_s * 1e3,
                "iterations": args.steps,
                "rollout_ms": ro[2] * 1e3, "rollout_env_steps_per_s": T * n_local / ro[2],
                "rollout_ms_unpipelined": ro[1] * 1e3, "host_env_step_ms": step_s * 1e3,
                "host_threads": henv.threads, "env_groups": 2,
                "pcie_bytes_per_vector_step": per_step_bytes,
                "note": f"{args.steps} iterations (as many as value's) with the envs stepped on the host: the C++ thread pool steps the "
                        "clean-room QuAntruped stand-in (not MuJoCo) into pinned buffers, pipelined over 2 env "
                        "groups (ddrl_rollout_hostenv: one group's host step overlaps the other's device work "
                        "and PCIe transfers); rollout_ms_unpipelined = the same with one group; host_env_step_ms "
                        "= one host step of all envs alone"}
        henv.close()

    upd_avg_ms = float(np.mean(upd_ms))
    steps_per_policy = int(steps_done[-1])
    mb_latency_ms = upd_avg_ms / steps_per_policy                 # one policy's sequential step
    mb_amortized_ms = upd_avg_ms / (steps_per_policy * P)        # reference's learn_time / (P*10*nb)
    d = cfg.obs_dim[0]
    rows_per_step = learner.rows_per_rank if ddp else 128
    flops_row = gnn_flops_per_row(A) if gnn else ffn_flops_per_row(d, A)
    flops_launch = flops_row * rows_per_step * steps_per_policy * P
    achieved_tf = flops_launch / (upd_avg_ms * 1e-3) / 1e12
    ks1 = (d + 3) // 4
    # the GNN gradient launch reduces over its tiles in its own tail when it covers a full
    # 128-row minibatch (32 tiles per combination) and the context runs the one-launch step
    # (gnn.hip launch_step_gnn: ga.tail) -- asked of the library, which may have turned it off
    # (DDRL_GNN_TAIL=0, occupancy / owner-list refusal, fallback after a failed step)
    gnn_tail = gnn and rows_per_step == 128 and (uctx or ctx).gnn_one_launch()
    pkey = pmc_key(args.env, gnn_tail)
    if gnn:
        if ddp:
            coll = "RCCL" if backend == "nccl" else backend
            kernel = (f"k_gnn<GRAD> (reduction in its tail) + {coll} all-reduce + k_apply_adam per minibatch step"
                      if gnn_tail else
                      f"k_gnn<GRAD> + k_gnn_reduce + {coll} all-reduce + k_apply_adam per minibatch step")
        else:
            kernel = ("k_gnn<GRAD> with the reduction and clip + Adam in its tail (one launch per minibatch step)"
                      if gnn_tail else "k_gnn<GRAD> + k_gnn_reduce + k_gnn_adam (three launches per minibatch step)")
        # (tiles of 4 graphs) x (actor, critic) x 4 backward shares (gnn.hip GNN_Z), one per CU
        active_cus = min(256, 2 * ((rows_per_step + 3) // 4) * 4)
        model = f"shared GraphNet/MPNN leg policy (4 nodes x 19 features + ego quaternion, A={A})"
    else:
        coll = "RCCL" if backend == "nccl" else backend
        kernel = (f"k_update_ffn<{A}, {ks1}> grad + {coll} all-reduce + k_apply_adam per step" if ddp else
                  "k_update_ffn (fused PPO minibatch SGD, one launch per iteration)")
        # the fused launch keeps 2 workgroups (policy / value branch) per policy, one per CU,
        # times the row split (DDRL_UPDATE_SPLIT, default 2); the data-parallel gradient launch
        # splits the same way when its rows fill both halves (capi.cpp grad_split: > 64 rows)
        split = 1 if os.environ.get("DDRL_UPDATE_SPLIT", "2") == "1" or (ddp and rows_per_step <= 64) else 2
        active_cus = 2 * P * split
        model = f"{P} {'shared' if P == 1 else 'independent'} fcnet 2x64 polic{'y' if P == 1 else 'ies'} (d={d}, A={A})"
    # algorithmic HBM bytes: each minibatch row's record fields read once per branch
    # (policy: obs, action, old logits, logp, adv; value: obs, vf, vt) + its shuffle index.
    # The fcnet launch keeps theta / Adam m, v on chip for the whole launch (LDS + registers),
    # so its per-step bytes are the records.  A GNN step is a launch of its own (one, with the
    # reduction and Adam in its tail), so every step also reads and writes theta, m, v (6 x 4 B
    # per parameter); where the summed gradient goes through memory (three launches, or the
    # data-parallel all-reduce) it is written and read once more (2 x 4 B per parameter)
    obs_len = 93 if gnn else d
    rec_bytes_launch = 4 * (2 * obs_len + 3 * A + 4 + 2) * rows_per_step * steps_per_policy * P
    if gnn:
        grad_io = 0 if (gnn_tail and not ddp) else 2
        rec_bytes_launch += (6 + grad_io) * 4 * ctx.n_params[0] * steps_per_policy * P
    ddp_how = ("RCCL all-reduce of the gradient every SGD step, loop in the library (ddrl_ppo_update_ddp)"
               if isinstance(learner, NativeDataParallelLearner) else
               f"{'RCCL' if backend == 'nccl' else backend} all-reduce of the gradient every SGD step, Python loop") \
        if ddp else ""
    coll_name = "RCCL" if backend == "nccl" else backend
    parallelism = (f"data-parallel over {world} ranks: {ddp_how} "
                   f"({args.ddp_mode} mode, {rows_per_step} rows per rank per step)" if ddp else
                   (f"gather over {world} ranks: every rank rolls out {n_local} envs, one {coll_name} all-gather "
                    f"of the records per iteration, the same fused update over the union batch of "
                    f"{n_local * world} envs on every rank (no per-step collective)" if gather else
                    "replicas (no collective)"))
    # provenance of the committed counter pass: its kernel's duration per
    # sequential step beside this run's; > 3 % apart marks `traffic` (and the MFMA-busy figures)
    # as from another build or box
    pmc_ns = None if ddp else pmc_ns_per_step(pkey, P)
    meas_ns = mb_latency_ms * 1e6
    # the same recipe's kernel-trace pass, when this run is the configuration it traced: one
    # dispatch per iteration's update (fcnet) or per step (GraphNet)
    comparable = (not ddp and not gather and args.envs == PROFILED_ENVS.get(pkey) and args.sgd_iter is None
                  and world == 1)
    trace_ns = trace_ns_per_step(pkey, 1 if gnn else steps_per_policy) if comparable else None
    stale = None if trace_ns is None else abs(trace_ns / meas_ns - 1.0) > 0.03
    result = {
        "metric": metric_name(args.envs),
        "value": env_steps / t_max,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": t_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic QuAntruped rollouts resident in HBM (no MuJoCo); Glorot-init weights",
        "config": {
            "workload": f"{args.env}: {args.envs} envs x {cfg.n_agents} leg agents, {model}, T={T}, "
                        f"train batch {R[0]} rows/policy/rank, {E} epochs x {steps_per_policy // E} "
                        f"minibatches x {rows_per_step} rows",
            "envs_total": args.envs, "envs_per_gpu": n_local, "parallelism": parallelism,
        },
        "ppo_update_ms_per_minibatch": mb_amortized_ms,
        "ppo_update_ms_per_minibatch_latency": mb_latency_ms,
        "update_kernel_ms": upd_avg_ms,
        "roofline": {
            "kernel": kernel,
            "bound": "mfma", "achieved": achieved_tf, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved_tf / PEAK_FP32_TFLOPS,
            "traffic": None if ddp else pmc_traffic(pkey, steps_per_policy * P),
            "traffic_source": None if ddp else f"{pmc_summary(pkey)[1]} [{pkey}] (bytes per step x steps of this update)",
            "pmc_kernel_ns_per_step": pmc_ns, "trace_kernel_ns_per_step": trace_ns,
            "measured_ns_per_step": meas_ns, "traffic_stale": stale,
            "algorithmic_flops_per_launch": flops_launch,
            "algorithmic_bytes_per_launch": rec_bytes_launch,
            "active_cus": active_cus,
            "frac_of_active_cus": achieved_tf / (PEAK_FP32_TFLOPS * active_cus / 256),
            **({} if ddp else pmc_mfma(pkey)),
        },
    }
    if pcie is not None:
        result["pcie_inclusive"] = pcie
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_envs = cpu_sample_envs(args.env, args.cpu_envs)
        v, dt, sample = cpu_baseline(args.env, cpu_envs, T)
        result["cpu_baseline"] = {"value": v, "unit": "env-steps/s", "cores": 1, "kind": "port",
                                  "sample": sample + f"; {dt:.1f} s", "host_cpus": os.cpu_count()}
        # the same sample on this job's share of the host cores (OMP_NUM_THREADS
        # on the GPU box; the machine's CPUs are shared between jobs), parallel over env chunks
        # (rollout) and over the independent policies (update), in a child process that never
        # touched the GPU (its worker pool forks)
        nthr = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count())
        import subprocess
        code = ("import json, bench; v, dt, w = bench.cpu_baseline_parallel(%r, %d, %d, %d); "
                "print(json.dumps([v, dt, w]))" % (args.env, cpu_envs, T, nthr))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=600,
                           cwd=os.path.dirname(os.path.abspath(__file__)))
        if r.returncode == 0:
            v2, dt2, w2 = json.loads(r.stdout.strip().splitlines()[-1])
            result["cpu_baseline_all_cores"] = {
                "value": v2, "unit": "env-steps/s", "cores": w2, "kind": "port",
                "sample": f"same sample on {w2} worker processes: rollout over env chunks, update over the "
                          f"{ctx.cfg.n_policies} polic{'y' if ctx.cfg.n_policies == 1 else 'ies'} (each "
                          f"policy's minibatch chain is sequential); {dt2:.1f} s"}
        else:
            result["cpu_baseline_all_cores"] = {"error": r.stderr[-300:]}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if uctx is not None:
        uctx.close()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
