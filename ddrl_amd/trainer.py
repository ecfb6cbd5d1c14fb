"""PPO trainer over the HIP hot path -- the drop-in for train_experiment_1's tune.run("PPO").

Reference call stack: RLlib PPOTrainer with ParallelRollouts ->
postprocess_ppo_gae -> StandardizeFields(["advantages"]) -> TrainTFMultiGPU (num_sgd_iter
epochs over R // sgd_minibatch_size shuffled minibatches per policy) -> update_kl.
Here one `train()` call is one training iteration: T = rollout_fragment_length vector env
steps on the device, bootstrap + GAE on the device, then one fused persistent update launch
for all policies (or, for a shared policy across ranks, per-minibatch gradient all-reduce).

The config dict uses the reference's keys (train_experiment_1_architecture_on_flat.py:96-168).
"""
from __future__ import annotations

import json
import math
import os
import time

import numpy as np

from . import native as N
from .spec import PPO_DEFAULTS, make_cfg


def glorot_ffn_flat(rng, d, A, hidden=64):
    """GlorotUniformScaled init (models/glorot_uniform_scaled_initializer.py:3-19): hidden
    kernels scale 1.0, fc_out / value_out scale 0.01, biases 0; Keras flat order."""
    def g(fi, fo, s):
        lim = math.sqrt(6.0 * s / (fi + fo))
        return rng.uniform(-lim, lim, size=(fi, fo)).astype(np.float32)
    z = lambda n: np.zeros(n, np.float32)
    parts = [g(d, hidden, 1.0), z(hidden), g(d, hidden, 1.0), z(hidden),
             g(hidden, hidden, 1.0), z(hidden), g(hidden, hidden, 1.0), z(hidden),
             g(hidden, 2 * A, 0.01), z(2 * A), g(hidden, 1, 0.01), z(1)]
    return np.concatenate([p.reshape(-1) for p in parts])


def leg_coupling_init(A):
    """LegCoupling.build (models/coupling_net_glorot_uniform_init.py:20): the table starts at
    [[1, 1], [-1, -1], [-1, -1], [1, 1]] (FL, HL, HR, FR), not at a random draw."""
    return np.resize(np.array([[1, 1], [-1, -1], [-1, -1], [1, 1]], np.float32), (4, A)).reshape(-1)


def rank_seeds(seed, rank):
    """(env seed, exploration-noise seed) of one rank: every rank samples its own trajectories
    (like RLlib's rollout workers, whose envs are seeded per worker index), while the weights
    come from `seed` alone and are identical on every rank.  Rank 0 keeps the single-process
    seeds."""
    return seed + 1_000_003 * rank, seed + 1 + 1_000_003 * rank


class PPOTrainer:
    """Multi-agent PPO on one device (one env shard).

    env_backend: an object with reset() -> obs[N, D] (device tensor) and
    step(actions[N, 8]) -> (obs_next, fw[N], cfrc[N, 14, 6], done[N] uint8); defaults to the
    synthetic vectorized QuAntruped (`ddrl_amd.envs.SyntheticVecEnv`).
    """

    def __init__(self, config, n_envs=None, device=0, env_backend=None, seed=0, stream=None):
        """Multi-process use: initialize torch.distributed first (one process per GPU).
        Shared-policy envs then train data-parallel (config "parallel": "ddp", the default
        for one policy; "ddp_mode": "split" | "local", see ddrl_amd.ddp); multi-policy envs
        run as independent replicas ("parallel": "replicas").  "parallel": "gather" (any env):
        every rank rolls out its own envs, the records of all ranks are all-gathered once per
        iteration into a learner context sized for the union batch, and every rank runs the
        same fused update over it with the same schedule -- weights identical on all ranks, no
        per-step collective (the union batch equals a single-process run over all envs)."""
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.config = {**PPO_DEFAULTS, **config}
        c = self.config
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        env = c["env"]
        self.n_envs = int(n_envs or c.get("num_envs", c.get("num_workers", 2) * c.get("num_envs_per_worker", 4)))
        self.T = int(c["rollout_fragment_length"])
        self.cfg, self.env = make_cfg(env, self.n_envs, self.T, c)
        torch.cuda.set_device(device)
        self.device = torch.device("cuda", device)
        self.stream = stream or torch.cuda.current_stream(self.device)
        self.ctx = N.Context(self.cfg, device, self.stream.cuda_stream)
        self.policy_ids = list(type(self.env).policy_names)
        P = self.cfg.n_policies
        self.rng = np.random.default_rng(seed)              # weights: identical on every rank
        self.sched_rng = np.random.default_rng(seed + 7919 * (self.rank + 1))
        env_seed, noise_seed = rank_seeds(seed, self.rank)  # trajectories: different on every rank
        for p in range(P):
            if self.cfg.model_kind == N.MODEL_FFN:
                theta = glorot_ffn_flat(self.rng, self.cfg.obs_dim[p], self.cfg.act_dim)
                if self.cfg.leg_coupling:
                    theta = np.concatenate([theta, leg_coupling_init(self.cfg.act_dim)])
                self.ctx.params_set(p, theta)
            else:
                from .models import glorot_gnn_flat
                layer = {v: k for k, v in N.GNN_LAYERS.items()}[self.cfg.gnn_layer]
                self.ctx.params_set(p, glorot_gnn_flat(self.rng, self.cfg.act_dim, layer=layer))
        self.kl_coeff = [float(c["kl_coeff"])] * P
        if env_backend is None and c.get("env_backend", "synthetic") == "host":
            # extension: the host env plane (the QuAntruped stand-in on host threads; TVel
            # target velocities drawn per env from env_config["target_velocity"] on every reset)
            from .envs import HostVecEnv
            env_backend = HostVecEnv(self.n_envs, self.cfg.obs_full_dim, self.device, seed=env_seed,
                                     n_threads=int(c.get("num_host_threads", 4)),
                                     target_velocity=self.env.target_velocity_list or 0.0)
        elif env_backend is None:
            from .envs import SyntheticVecEnv
            env_backend = SyntheticVecEnv(self.n_envs, self.cfg.obs_full_dim, self.device, seed=env_seed)
        self.backend = env_backend
        self.actions = torch.zeros((self.n_envs, 8), dtype=torch.float32, device=self.device)
        self.noise_gen = torch.Generator(device=self.device)
        self.noise_gen.manual_seed(noise_seed)
        self.timesteps_total = 0
        self.iteration = 0
        self.parallel = c.get("parallel") or ("ddp" if self.world > 1 and P == 1 else "replicas")
        if self.parallel not in ("ddp", "replicas", "gather"):
            raise ValueError(f"parallel {self.parallel!r}: 'ddp', 'replicas' or 'gather'")
        self.rctx = self.ctx   # the rollout context (the learner's own, except in "gather" mode)
        if self.parallel == "gather":
            from .ddp import Comm
            self.comm = Comm(self.device if self.world > 1 and dist.get_backend() == "nccl" else "cpu") \
                if self.world > 1 else None
            ucfg, _ = make_cfg(env, self.n_envs * self.world, self.T, c)
            self.ctx = N.Context(ucfg, device, self.stream.cuda_stream)   # learner: union batch
            for p in range(P):
                self.ctx.params_set(p, self.rctx.params_get(p))
            self.pfilter_base = ([self.rctx.policy_filter_get(p) for p in range(P)]
                                 if self.cfg.policy_filter else None)
            self.rctx.policy_filter_delta_reset()
            self.sched_rng = np.random.default_rng(seed + 7919)   # the same schedule on every rank
        if self.parallel == "ddp":
            from .ddp import (Comm, DataParallelLearner, HipBackend, NativeDataParallelLearner, PeerLearner,
                              native_comm_init)
            rccl = dist.get_backend() == "nccl"
            self.comm = Comm(self.device if rccl else "cpu")
            loop = c.get("ddp_loop", "native")
            if loop == "peer":
                # extension: the two ranks' update as one fused launch split across them; only for
                # what ddrl_peer_attach supports, otherwise the all-reduce learner
                why = [w for w, bad in (("a GraphNet model", self.cfg.model_kind != N.MODEL_FFN),
                                        (f"{self.world} ranks (peer mode pairs exactly two)", self.world != 2),
                                        (f"sgd_minibatch_size {self.cfg.sgd_minibatch_size} (not 128)",
                                         self.cfg.sgd_minibatch_size != 128),
                                        ("DDRL_UPDATE_SPLIT=1 (peer mode needs the row split)",
                                         os.environ.get("DDRL_UPDATE_SPLIT") == "1")) if bad]
                if why:
                    import warnings
                    warnings.warn(f"ddp_loop 'peer' does not support {', '.join(why)}: using the all-reduce "
                                  "data-parallel learner")
                    loop = "native" if rccl else "python"
            if loop == "peer":
                self.learner = PeerLearner(self.ctx, self.comm, 0, self.cfg.sgd_minibatch_size)
            elif rccl and loop == "native":
                native_comm_init(self.ctx, self.comm)
                self.learner = NativeDataParallelLearner(self.ctx, self.comm, 0, self.cfg.sgd_minibatch_size,
                                                         c.get("ddp_mode", "split"))
            else:
                self.learner = DataParallelLearner(HipBackend(self.ctx), self.comm, 0, self.cfg.sgd_minibatch_size,
                                                   c.get("ddp_mode", "split"))
            self.filter_base = self.ctx.filter_get()
            self.ctx.filter_delta_reset()
            self.pfilter_base = ([self.ctx.policy_filter_get(p) for p in range(P)]
                                 if self.cfg.policy_filter else None)
            self.ctx.policy_filter_delta_reset()
            self.grad = torch.zeros(self.ctx.n_params[0], dtype=torch.float32, device=self.device)
        self.workers = _Workers(self)
        self.rctx.observe(self.backend.reset())

    # -- one iteration ---------------------------------------------------------------
    def _sample(self):
        torch, cfg = self.torch, self.cfg
        rctx = self.rctx
        for t in range(self.T):
            eps = torch.randn((self.n_envs, cfg.n_agents, cfg.act_dim), device=self.device,
                              generator=self.noise_gen)
            rctx.act(t, eps, self.actions)
            obs, fw, cfrc, done = self.backend.step(self.actions)
            rctx.reward(t, fw, cfrc, self.actions, done)
            rctx.observe(obs)
        rctx.bootstrap()
        rctx.gae()
        if self.parallel == "gather":
            from .ddp import sync_filters, sync_standardize, standardize_constants
            for p in range(self.cfg.n_policies):
                if self.pfilter_base is not None:   # RLlib synchronize_filters
                    d = rctx.policy_filter_get(p, delta=True)
                    self.pfilter_base[p] = (sync_filters(self.comm, self.pfilter_base[p], d) if self.comm else
                                            sync_filters_local(self.pfilter_base[p], d))
                    rctx.policy_filter_set(p, *self.pfilter_base[p])
                    self.ctx.policy_filter_set(p, *self.pfilter_base[p])
                sums = rctx.adv_sums_get(p)
                norm = sync_standardize(self.comm, sums) if self.comm else standardize_constants(sums)
                self.ctx.adv_norm_set(p, *norm)
            rctx.policy_filter_delta_reset()
            return
        if self.parallel == "ddp":
            from .ddp import sync_filters, sync_standardize
            # The env-side MeanStdFilter is a per-process singleton in the reference
            # (simulation_envs/observation_filter.py:3-12) that RLlib never synchronizes: it stays
            # rank-local unless the config asks for a merged one ("sync_env_filter": True, an
            # extension).  RLlib's per-policy filters are synchronized (synchronize_filters).
            if self.config.get("sync_env_filter", False):
                merged = sync_filters(self.comm, self.filter_base, self.ctx.filter_delta_get())
                self.ctx.filter_set(*merged)
                self.ctx.filter_delta_reset()
                self.filter_base = merged
            if self.pfilter_base is not None:   # RLlib synchronize_filters for the policy filters
                for p in range(self.cfg.n_policies):
                    self.pfilter_base[p] = sync_filters(self.comm, self.pfilter_base[p],
                                                        self.ctx.policy_filter_get(p, delta=True))
                    self.ctx.policy_filter_set(p, *self.pfilter_base[p])
                self.ctx.policy_filter_delta_reset()
            for p in range(self.cfg.n_policies):
                self.ctx.adv_norm_set(p, *sync_standardize(self.comm, self.ctx.adv_sums_get(p)))

    def _schedule(self, p):
        """SampleBatch.shuffle() + one permutation of the minibatch slots per epoch."""
        R = self.T * self.ctx.layout[p]["C"]
        mb = self.cfg.sgd_minibatch_size
        shuffle = self.sched_rng.permutation(R).astype(np.int32)
        nb = max(1, R // mb)
        perms = np.stack([self.sched_rng.permutation(nb) for _ in range(self.cfg.num_sgd_iter)]).astype(np.int32)
        return shuffle, perms, nb

    def _learn_ddp(self):
        torch = self.torch
        R = self.T * self.ctx.layout[0]["C"]
        shuffle, perms = self.learner.schedule(self.sched_rng, R, self.cfg.num_sgd_iter)
        kl = self.learner.learn(torch.from_numpy(shuffle).to(self.device), perms, self.kl_coeff[0], self.grad)
        nb = perms.shape[1]
        last = self.ctx.ppo_stats(0, nb, self.learner.stats_first).astype(np.float64).mean(0)
        pid = self.policy_ids[0]
        learner = {pid: {"cur_kl_coeff": float(np.float32(self.kl_coeff[0])),
                         "cur_lr": float(np.float32(self.cfg.lr)), "total_loss": last[0],
                         "policy_loss": last[1], "vf_loss": last[2], "kl": kl, "entropy": last[4],
                         "vf_explained_var": last[5], "entropy_coeff": self.cfg.entropy_coeff,
                         "num_ranks": self.world}}
        self.kl_coeff[0] = update_kl(self.kl_coeff[0], kl, self.config["kl_target"])
        return learner

    def _gather_records(self):
        """All-gather every rank's records (rank-major) into the learner context's union batch."""
        from .ddp import gather_records
        for p in range(self.cfg.n_policies):
            gather_records(self.comm, self.rctx.records_tensor(p), self.ctx.records_tensor(p))

    def _learn(self):
        if self.parallel == "ddp":
            return self._learn_ddp()
        if self.parallel == "gather":
            self._gather_records()
        torch = self.torch
        P = self.cfg.n_policies
        sh, pe, nbs = [], [], []
        for p in range(P):
            s, q, nb = self._schedule(p)
            sh.append(torch.from_numpy(s).to(self.device))
            pe.append(torch.from_numpy(q).to(self.device))
            nbs.append(nb)
        self.ctx.ppo_update((1 << P) - 1, sh, pe, self.kl_coeff)
        learner = {}
        for p, pid in enumerate(self.policy_ids):
            st = self.ctx.ppo_stats(p, nbs[p], first=(self.cfg.num_sgd_iter - 1) * nbs[p])
            last = st.astype(np.float64).mean(0)   # TrainTFMultiGPU: last epoch's mean
            learner[pid] = {"cur_kl_coeff": float(np.float32(self.kl_coeff[p])),
                            "cur_lr": float(np.float32(self.cfg.lr)),
                            "total_loss": last[0], "policy_loss": last[1], "vf_loss": last[2],
                            "kl": last[3], "entropy": last[4], "vf_explained_var": last[5],
                            "grad_gnorm": last[6], "entropy_coeff": self.cfg.entropy_coeff}
            self.kl_coeff[p] = update_kl(self.kl_coeff[p], last[3], self.config["kl_target"])
        if self.parallel == "gather":   # the next rollout uses the updated weights
            for p in range(P):
                self.rctx.params_set(p, self.ctx.params_get(p))
        return learner

    def train(self):
        torch = self.torch
        t0 = time.perf_counter()
        self._sample()
        torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        learner = self._learn()
        t2 = time.perf_counter()
        steps = self.T * self.n_envs
        self.timesteps_total += steps
        self.iteration += 1
        cb = self.config.get("callbacks", {}).get("on_train_result") if isinstance(
            self.config.get("callbacks"), dict) else None
        self.last_learner = learner
        result = {"training_iteration": self.iteration, "timesteps_total": self.timesteps_total,
                  "timesteps_this_iter": steps, "info": {"learner": learner},
                  "timers": {"sample_time_ms": (t1 - t0) * 1e3, "learn_time_ms": (t2 - t1) * 1e3,
                             "sample_throughput": steps / (t1 - t0),
                             "learn_throughput": steps / (t2 - t1)}}
        if cb:
            cb({"result": result, "trainer": self})
        return result

    # -- state -------------------------------------------------------------------------
    def get_weights(self):
        return {pid: self.ctx.params_get(p) for p, pid in enumerate(self.policy_ids)}

    def set_weights(self, weights):
        """Writes the learner context and, in "gather" mode, the rollout context too: the next
        fragment must be sampled (and its logp / vf recorded) with the weights it trains."""
        for p, pid in enumerate(self.policy_ids):
            if pid in weights:
                self.ctx.params_set(p, weights[pid])
                if self.rctx is not self.ctx:
                    self.rctx.params_set(p, weights[pid])

    def save(self, path):
        """Checkpoint: weights, Adam m/v/beta powers, KL coefficients, filter state (npz,
        no pickle)."""
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        arrs = {}
        for p, pid in enumerate(self.policy_ids):
            m, v, b1, b2 = self.ctx.adam_get(p)
            arrs[f"{pid}/weights"] = self.ctx.params_get(p)
            arrs[f"{pid}/adam_m"], arrs[f"{pid}/adam_v"] = m, v
            arrs[f"{pid}/beta_powers"] = np.array([b1, b2], np.float32)
            arrs[f"{pid}/kl_coeff"] = np.array([self.kl_coeff[p]])
        n, M, S = self.rctx.filter_get()   # the env-side filter lives where the rollout runs
        arrs["filter/n"], arrs["filter/M"], arrs["filter/S"] = np.array([n]), M, S
        if self.cfg.policy_filter:
            for p, pid in enumerate(self.policy_ids):
                n, M, S = self.ctx.policy_filter_get(p)
                arrs[f"{pid}/filter/n"], arrs[f"{pid}/filter/M"], arrs[f"{pid}/filter/S"] = np.array([n]), M, S
        arrs["meta"] = np.frombuffer(json.dumps({"iteration": self.iteration,
                                                 "timesteps_total": self.timesteps_total}).encode(), np.uint8)
        np.savez(path, **arrs)
        return path

    def restore(self, path):
        z = np.load(path, allow_pickle=False)
        for p, pid in enumerate(self.policy_ids):
            self.ctx.params_set(p, z[f"{pid}/weights"])
            if self.rctx is not self.ctx:
                self.rctx.params_set(p, z[f"{pid}/weights"])
            b = z[f"{pid}/beta_powers"]
            self.ctx.adam_set(p, z[f"{pid}/adam_m"], z[f"{pid}/adam_v"], float(b[0]), float(b[1]))
            self.kl_coeff[p] = float(z[f"{pid}/kl_coeff"][0])
        self.rctx.filter_set(float(z["filter/n"][0]), z["filter/M"], z["filter/S"])
        if self.cfg.policy_filter:
            for p, pid in enumerate(self.policy_ids):
                for cx in {id(self.ctx): self.ctx, id(self.rctx): self.rctx}.values():
                    cx.policy_filter_set(p, float(z[f"{pid}/filter/n"][0]), z[f"{pid}/filter/M"],
                                         z[f"{pid}/filter/S"])
        meta = json.loads(bytes(z["meta"]).decode())
        self.iteration, self.timesteps_total = meta["iteration"], meta["timesteps_total"]
        self._after_load({})

    def _after_load(self, learner):
        """State that follows a restore: the learner statistics that belong to the restored
        weights (none for an npz checkpoint, the file's own for an RLlib one), and, for the
        data-parallel / gather modes, the base of the per-policy filter sync, which must be the
        restored RunningStat (else the next sync merges the delta into the stale base)."""
        self.last_learner = learner
        if self.parallel in ("ddp", "gather") and getattr(self, "pfilter_base", None) is not None:
            self.pfilter_base = [self.ctx.policy_filter_get(p) for p in range(self.cfg.n_policies)]
            self.rctx.policy_filter_delta_reset()

    def restore_rllib(self, path):
        """Load a published RLlib checkpoint (Results/**/checkpoint-1250, the file
        evaluation/evaluate_trained_policies_pd.py:93-96 restores): per policy the Keras-order
        weights, Adam m / v and beta powers, the RLlib MeanStdFilter RunningStat (when this
        trainer runs observation_filter = MeanStdFilter) and the KL coefficient.  Read with the
        no-code reader (ddrl_amd.rllib_checkpoint: a pickletools opcode walk; nothing in the
        file is executed).  Returns the policy ids loaded."""
        from .rllib_checkpoint import policy_ids, policy_state, read_checkpoint
        ck = read_checkpoint(path)
        return self.load_policy_states({pid: policy_state(ck, pid) for pid in policy_ids(ck)})

    def rllib_policy_states(self):
        """Per policy id the state rllib_checkpoint.worker_tree writes: Keras-order weights,
        Adam m / v, beta powers, the RLlib MeanStdFilter RunningStat (when this trainer runs
        observation_filter = MeanStdFilter; NoFilter otherwise) and the variable shapes."""
        from .rllib_checkpoint import ffn_shapes, gnn_shapes
        out = {}
        A = self.cfg.act_dim
        for p, pid in enumerate(self.policy_ids):
            m, v, b1, b2 = self.ctx.adam_get(p)
            d = int(self.cfg.obs_dim[p])
            if self.cfg.model_kind == N.MODEL_FFN:
                shapes = ffn_shapes(d, 2 * A) + ([("leg_coupling", (4, A))] if self.cfg.leg_coupling else [])
            else:
                shapes = gnn_shapes(2 * A, layer={v: k for k, v in N.GNN_LAYERS.items()}[self.cfg.gnn_layer])
            st = {"weights": self.ctx.params_get(p), "adam_m": m, "adam_v": v,
                  "beta_powers": (np.float32(b1), np.float32(b2)), "shapes": shapes, "obs_dim": d,
                  "filter": None, "filter_buffer": None}
            if self.cfg.policy_filter:
                st["filter"] = self.ctx.policy_filter_get(p)
            else:
                st["filter_kind"] = "NoFilter"
            out[pid] = st
        return {pid: out[pid] for pid in sorted(out)}   # Ray 1.0.1 writes the policies sorted by id

    def save_rllib(self, checkpoint_dir, time_total=0.0, episodes_total=0):
        """Write an RLlib (Ray 1.0.1) checkpoint of this trainer --
        <checkpoint_dir>/checkpoint_<i>/checkpoint-<i> + .tune_metadata -- in the layout
        PPOTrainer.restore reads (evaluation/evaluate_trained_policies_pd.py:93-96), with the
        learner statistics of the last train() call.  The writer emits the pickle opcodes
        itself (ddrl_amd.rllib_checkpoint.emit); it reproduces every published checkpoint
        byte for byte from its contents (tests/test_checkpoint.py)."""
        from .rllib_checkpoint import write_checkpoint
        last = getattr(self, "last_learner", {}) or {}
        learner = {}
        for p, pid in enumerate(self.policy_ids):
            s = dict(last.get(pid, {}))
            # no statistics for the current weights (no train() since the trainer was built or
            # restored from an npz file): the row carries the current coefficient and no "kl",
            # so a reload keeps the coefficient as it is (load_policy_states runs update_kl only
            # with a kl)
            s.setdefault("cur_kl_coeff", float(np.float32(self.kl_coeff[p])))
            s.setdefault("cur_lr", float(np.float32(self.cfg.lr)))
            s.setdefault("entropy_coeff", float(self.cfg.entropy_coeff))
            learner[pid] = s
        return write_checkpoint(checkpoint_dir, self.iteration, self.rllib_policy_states(), learner,
                                self.timesteps_total, time_total=time_total, episodes_total=episodes_total)

    def load_policy_states(self, states):
        """Per policy id: {"weights", "adam_m", "adam_v", "beta_powers", "filter" (n, M, S) or
        None, "kl_coeff" or None} (ddrl_amd.rllib_checkpoint.policy_state's layout) into the
        context; returns the policy ids loaded."""
        missing = [pid for pid in self.policy_ids if pid not in states]
        learner = {}
        if missing:
            raise ValueError(f"checkpoint has policies {sorted(states)}, this env needs {self.policy_ids}")
        for p, pid in enumerate(self.policy_ids):
            st = states[pid]
            if st["weights"].size != self.ctx.n_params[p]:
                raise ValueError(f"{pid}: checkpoint holds {st['weights'].size} parameters, the model "
                                 f"{self.ctx.n_params[p]}")
            self.ctx.params_set(p, st["weights"])
            self.ctx.adam_set(p, st["adam_m"], st["adam_v"], *st["beta_powers"])
            if self.cfg.policy_filter and st["filter"] is not None:
                self.ctx.policy_filter_set(p, *st["filter"])
                self.rctx.policy_filter_set(p, *st["filter"])
            if self.rctx is not self.ctx:
                self.rctx.params_set(p, st["weights"])
            stats = dict(st.get("learner_stats") or {})
            if self.config.get("restore_kl_coeff", "checkpoint") == "config":
                # RLlib 1.0.1: the TF policy state holds only model and optimizer variables
                # (KLCoeffMixin has no get_state), so PPOTrainer.restore starts again from
                # config["kl_coeff"]
                self.kl_coeff[p] = float(self.config["kl_coeff"])
                stats.pop("kl", None)
                stats["cur_kl_coeff"] = self.kl_coeff[p]
            elif st["kl_coeff"] is not None:
                # extension: continue from the file's coefficient.  Its
                # cur_kl_coeff is the coefficient the checkpointed iteration trained with; the
                # next iteration's is update_kl of it and that iteration's kl (RLlib runs update_kl
                # after the learner step, ppo.py UpdateKL)
                kl = stats.get("kl")
                self.kl_coeff[p] = (update_kl(st["kl_coeff"], kl, self.config["kl_target"]) if kl is not None
                                    else st["kl_coeff"])
                stats["cur_kl_coeff"] = st["kl_coeff"]
            learner[pid] = stats
        self._after_load(learner)
        return list(self.policy_ids)

    def stop(self):
        if self.rctx is not self.ctx:
            self.rctx.close()
        self.ctx.close()
        if hasattr(self.backend, "close"):
            self.backend.close()


class _EnvHandle:
    """What `worker.foreach_env(fn)` hands to fn: the env spec (the reference's MultiAgentEnv
    class surface), whose update_environment_after_epoch also resets the vectorized backend's
    envs (quantruped_adaptor_multi_environment.py:97-122: update_after_epoch, then env.reset())."""

    def __init__(self, trainer):
        self._trainer = trainer

    def update_environment_after_epoch(self, timesteps_total):
        self._trainer.env.update_environment_after_epoch(timesteps_total)
        hook = getattr(self._trainer.backend, "update_environment_after_epoch", None)
        if hook is not None:
            hook(timesteps_total)

    def __getattr__(self, name):
        return getattr(self._trainer.env, name)


class _Worker:
    def __init__(self, trainer):
        self._trainer = trainer

    def foreach_env(self, fn):
        """RolloutWorker.foreach_env: fn over this worker's envs -- one vectorized env here."""
        return [fn(_EnvHandle(self._trainer))]


class _Workers:
    """trainer.workers (RLlib WorkerSet) for the callbacks the reference's training scripts
    install: train_experiment_1_architecture_on_flat.py:171-178 runs
    trainer.workers.foreach_worker(lambda ev: ev.foreach_env(lambda env:
    env.update_environment_after_epoch(timesteps))) after every iteration."""

    def __init__(self, trainer):
        self._trainer = trainer

    def foreach_worker(self, fn):
        return [fn(_Worker(self._trainer))]


def sync_filters_local(base, delta):
    from .ddp import merge_running_stats
    return merge_running_stats(base, [delta])


def update_kl(kl_coeff, sampled_kl, kl_target=0.01):
    """RLlib PPO update_kl (ppo_tf_policy.KLCoeffMixin)."""
    if sampled_kl > 2.0 * kl_target:
        return kl_coeff * 1.5
    if sampled_kl < 0.5 * kl_target:
        return kl_coeff * 0.5
    return kl_coeff


def run(config, stop=None, n_envs=None, device=0, verbose=True):
    """tune.run("PPO", config=config, stop={"timesteps_total": ...}) for one trial."""
    stop = stop or {"training_iteration": 1}
    tr = PPOTrainer(config, n_envs=n_envs, device=device)
    results = []
    while True:
        r = tr.train()
        results.append(r)
        if verbose:
            print(json.dumps({k: r[k] for k in ("training_iteration", "timesteps_total", "timers")}))
        if any(r.get(k, 0) >= v for k, v in stop.items()):
            break
    tr.stop()
    return results
