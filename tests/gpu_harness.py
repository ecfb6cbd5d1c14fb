"""Shared helpers for the GPU parity tests: build a context, run an oracle rollout on the
same seeded inputs, and compare record buffers."""
from __future__ import annotations

import numpy as np

from oracle import ddrl_oracle as O
from ddrl_amd import native as N
from ddrl_amd.spec import make_cfg


def make_ctx(env, n_envs, T, config=None, stream=None):
    import torch
    cfg, inst = make_cfg(env, n_envs, T, config)
    ctx = N.Context(cfg, 0, stream if stream is not None else torch.cuda.current_stream().cuda_stream)
    return ctx, cfg, inst


def policy_tables(cfg, inst):
    """Per policy: list of (slot -> agent name) and d, from the cfg the kernels use."""
    agents = list(inst.agent_names)
    out = []
    for p in range(cfg.n_policies):
        slots = [a for j, a in enumerate(agents) if cfg.agent_policy[j] == p]
        out.append(slots)
    return out


def init_params(ctx, cfg, seed, head_scale=30.0):
    rng = np.random.default_rng(seed)
    params = []
    for p in range(cfg.n_policies):
        A = cfg.act_dim
        pr = O.ffn_init(rng, cfg.obs_dim[p], 2 * A)
        pr["fc_out/kernel"] *= head_scale
        pr["value_out/kernel"] *= head_scale
        pr["fc_1/bias"] += rng.normal(size=64).astype(np.float32) * 0.1
        pr["fc_out/bias"] += np.concatenate([np.zeros(A), -0.5 * np.ones(A)]).astype(np.float32)
        shapes = O.ffn_param_shapes(cfg.obs_dim[p], 2 * A)
        ctx.params_set(p, O.pack(pr, shapes))
        params.append(pr)
    return params


class OracleRollout:
    """Oracle restatement of observe/act/reward/bootstrap/GAE for a vectorized env."""

    def __init__(self, cfg, inst, params, filt):
        self.cfg, self.inst, self.params = cfg, inst, params
        self.rs = O.RunningStat((cfg.obs_full_dim,))
        self.rs.n, self.rs.M[:], self.rs.S[:] = filt
        self.slots = policy_tables(cfg, inst)
        self.agents = list(inst.agent_names)
        T, N_ = cfg.frag_len, cfg.n_envs
        self.rec = []
        for p in range(cfg.n_policies):
            C = N_ * len(self.slots[p])
            self.rec.append(dict(obs=np.zeros((T, C, cfg.obs_dim[p]), np.float32),
                                 act=np.zeros((T, C, cfg.act_dim), np.float32),
                                 logits=np.zeros((T, C, 2 * cfg.act_dim), np.float32),
                                 logp=np.zeros((T, C), np.float32), vf=np.zeros((T, C), np.float32),
                                 rew=np.zeros((T, C), np.float32)))
        self.done = np.zeros((T, N_), np.uint8)
        self.stage = None
        # RLlib per-policy MeanStdFilter (observation_filter), unclipped, on the fp64 routed rows
        self.pf = ([O.RunningStat((cfg.obs_dim[p],)) for p in range(cfg.n_policies)]
                   if getattr(cfg, "policy_filter", 0) else None)

    def observe(self, obs, bounds=None):
        """bounds: env ranges observed by separate calls (ddrl_observe_range), each one filter
        push + normalization of its own rows; default one call over all envs."""
        bounds = [0, obs.shape[0]] if bounds is None else bounds
        parts = [self._observe_block(obs[a:b]) for a, b in zip(bounds[:-1], bounds[1:])]
        self.stage = [np.concatenate([pp[i] for pp in parts]) for i in range(len(parts[0]))]

    def _observe_block(self, obs):
        normed = O.mean_std_filter(obs, self.rs, update=True, clip=self.cfg.filter_clip)
        stage = []
        tables = self.model_tables()
        # gather columns; the constants -1 / -2 (LegID one-hot) become 0 / 1
        ext = np.concatenate([normed, np.zeros((normed.shape[0], 1)), np.ones((normed.shape[0], 1))], 1)
        col = lambda i: i if i >= 0 else normed.shape[1] + (-1 - i)
        for p in range(self.cfg.n_policies):
            cols = [ext[:, [col(i) for i in tables[a]]] for a in self.slots[p]]
            x = np.stack(cols, 1).reshape(-1, self.cfg.obs_dim[p])   # c = e * k + slot
            if self.pf is not None:
                x = O.mean_std_filter(x, self.pf[p], update=True, clip=None)
            stage.append(x.astype(np.float32))
        return stage

    def model_tables(self):
        return getattr(self.inst, "policy_obs_indices", self.inst.obs_indices)

    def forward(self, p, x):
        return O.ffn_forward(self.params[p], x)

    def act(self, t, eps):
        cfg = self.cfg
        A = cfg.act_dim
        actions = np.zeros((cfg.n_envs, 8), np.float32)
        for p in range(cfg.n_policies):
            x = self.stage[p]
            logits, value, _ = self.forward(p, x)
            k = len(self.slots[p])
            e_idx = [self.agents.index(a) for a in self.slots[p]]
            ep = eps[:, e_idx, :].reshape(-1, A)
            a = O.dg_sample(logits, ep)
            r = self.rec[p]
            r["obs"][t], r["act"][t], r["logits"][t] = x, a, logits
            r["logp"][t], r["vf"][t] = O.dg_logp(logits, a), value
            for s, name in enumerate(self.slots[p]):
                sign = np.where(getattr(self.inst, "action_negate", {}).get(name, [False] * A), -1.0, 1.0)
                actions[:, self.inst.action_indices[name]] = np.clip(a.reshape(-1, k, A)[:, s], -1, 1) * sign
        return actions

    def reward(self, t, fw, cfrc, actions, done):
        cfg = self.cfg
        for e in range(cfg.n_envs):
            ad = {a: actions[e, self.inst.action_indices[a]].astype(np.float64) for a in self.agents}
            tables = {a: (self.inst.contact_force_indices[a][0], self.inst.contact_force_indices[a][1])
                      for a in self.agents}
            if self.inst.reward_mode == "global":
                rw = O.global_reward(float(fw[e]), cfrc[e].astype(np.float64), ad,
                                     cfg.ctrl_cost_weight, cfg.contact_cost_weight)
            else:
                rw = O.per_leg_reward(float(fw[e]), cfrc[e].astype(np.float64), ad, tables,
                                      cfg.ctrl_cost_weight, cfg.contact_cost_weight,
                                      norm_reward=self.inst.reward_mode == "norm")
            for p in range(cfg.n_policies):
                k = len(self.slots[p])
                for s, a in enumerate(self.slots[p]):
                    self.rec[p]["rew"][t, e * k + s] = rw[a]
        self.done[t] = done

    def bootstrap(self):
        self.last_v = [self.forward(p, self.stage[p])[1] for p in range(self.cfg.n_policies)]

    def gae(self):
        out = []
        for p in range(self.cfg.n_policies):
            k = len(self.slots[p])
            dones = np.repeat(self.done, k, axis=1)
            adv, vt = O.gae_fragment(self.rec[p]["rew"], self.rec[p]["vf"], dones, self.last_v[p],
                                     self.cfg.gamma, self.cfg.lambda_)
            self.rec[p]["adv"], self.rec[p]["vt"] = adv, vt
            _, mean, std = O.standardize(adv.reshape(-1))
            out.append((mean, max(np.float32(1e-4), std)))
        return out

    def flat_records(self, p, lay):
        r = self.rec[p]
        T, C = r["vf"].shape
        out = np.zeros((T * C, lay["stride"]), np.float32)
        d = r["obs"].shape[-1]
        A = r["act"].shape[-1]
        out[:, lay["obs"]:lay["obs"] + d] = r["obs"].reshape(T * C, d)
        out[:, lay["act"]:lay["act"] + A] = r["act"].reshape(T * C, A)
        out[:, lay["logit"]:lay["logit"] + 2 * A] = r["logits"].reshape(T * C, 2 * A)
        for key, off in (("logp", "logp"), ("vf", "vf"), ("rew", "rew"), ("adv", "adv"), ("vt", "vt")):
            if key in r:
                out[:, lay[off]] = r[key].reshape(-1)
        if lay.get("leg", -1) >= 0:   # "cup": leg index of the row = slot (c = e * k + slot)
            out[:, lay["leg"]] = np.tile(np.arange(C) % len(self.slots[p]), T)
        return out


def synthetic_inputs(rng, cfg, T):
    N_ = cfg.n_envs
    obs = (rng.normal(size=(T + 1, N_, cfg.obs_full_dim)) * 2 + 0.5).astype(np.float32)
    eps = rng.normal(size=(T, N_, cfg.n_agents, cfg.act_dim)).astype(np.float32)
    fw = rng.normal(size=(T, N_)).astype(np.float32)
    cfrc = (rng.normal(size=(T, N_, 14, 6)) * 1.5).astype(np.float32)
    done = (rng.random(size=(T, N_)) < 0.05).astype(np.uint8)
    return obs, eps, fw, cfrc, done


def run_rollout(ctx, cfg, inst, params, rng, filt, T, orc_cls=None, pfilt=None):
    """Run the HIP rollout and the oracle on the same inputs; returns (oracle, inputs).
    pfilt: optional per-policy RLlib filter states [(n, M, S)] (cfg.policy_filter)."""
    import torch
    obs, eps, fw, cfrc, done = synthetic_inputs(rng, cfg, T)
    ctx.filter_set(*filt)
    orc = (orc_cls or OracleRollout)(cfg, inst, params, filt)
    if pfilt is not None:
        for p, (n, M, S) in enumerate(pfilt):
            ctx.policy_filter_set(p, n, M, S)
            orc.pf[p].n, orc.pf[p].M[:], orc.pf[p].S[:] = n, M, S
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    actions = torch.zeros((cfg.n_envs, 8), dtype=torch.float32, device="cuda")
    acts_gpu = []
    acts_orc = []
    for t in range(T):
        o_t = dev(obs[t])
        ctx.observe(o_t)
        orc.observe(obs[t])
        e_t = dev(eps[t])
        ctx.act(t, e_t, actions)
        a_orc = orc.act(t, eps[t])
        acts_gpu.append(actions.cpu().numpy().copy())
        acts_orc.append(a_orc)
        f_t, c_t, d_t = dev(fw[t]), dev(cfrc[t]), dev(done[t])
        # the env consumes the HIP actions; the oracle uses its own (compared separately)
        ctx.reward(t, f_t, c_t, actions, d_t)
        orc.reward(t, fw[t], cfrc[t], a_orc, done[t])
    ctx.observe(dev(obs[T]))
    orc.observe(obs[T])
    ctx.bootstrap()
    orc.bootstrap()
    ctx.gae()
    norms = orc.gae()
    torch.cuda.synchronize()
    return orc, norms, np.stack(acts_gpu), np.stack(acts_orc)


# --------------------------------------------------------------------------------------
# "cup" (SharedDecentralLegID env + leg-coupling fcnet): one shared leg policy, 4 rows per
# env, leg index = slot; the model input is the 19 features (no one-hot columns).
# --------------------------------------------------------------------------------------
CUP_ENV = "QuantrupedMultiEnv_SharedDecentralLegID"
CUP_CONFIG = {"model": {"custom_model": "cup"}}


def init_cup_params(ctx, cfg, seed, head_scale=30.0, perturb=True):
    rng = np.random.default_rng(seed)
    A, d = cfg.act_dim, cfg.obs_dim[0]
    pr = O.cup_init(rng, d, A)
    pr["fc_out/kernel"] *= head_scale
    pr["value_out/kernel"] *= head_scale
    pr["fc_1/bias"] += rng.normal(size=64).astype(np.float32) * 0.1
    pr["fc_out/bias"] += np.concatenate([np.zeros(A), -0.5 * np.ones(A)]).astype(np.float32)
    if perturb:   # off the +-1 start so that every coupling entry scales differently
        pr["leg_coupling"] = (pr["leg_coupling"] * rng.uniform(0.5, 1.5, size=(4, A))).astype(np.float32)
    ctx.params_set(0, O.pack(pr, O.cup_param_shapes(d, A)))
    return [pr]


class CupOracleRollout(OracleRollout):
    def model_tables(self):
        return self.inst.obs_indices

    def forward(self, p, x):
        leg = np.arange(x.shape[0]) % len(self.slots[p])
        return O.cup_forward(self.params[p], x, leg)


# --------------------------------------------------------------------------------------
# GraphNet ("gnn", DecentralShared_Graph): one shared leg policy, 4 rows per env (node n
# = agent n), record obs field = X [4][23] flattened + node index.
# --------------------------------------------------------------------------------------
GNN_ENV = "QuantrupedMultiEnv_DecentralShared_Graph"


def init_gnn_params(ctx, seed, head_scale=1.0, A=2, layer="mpnn"):
    rng = np.random.default_rng(seed)
    p = O.gnn_init(rng, 2 * A, layer=layer)
    for net in ("actor/", "critic/"):
        p[net + "linear_out/kernel"] *= head_scale
        p[net + "state_enc/bias"] += (rng.normal(size=p[net + "state_enc/bias"].shape) * 0.2).astype(np.float32)
    p["actor/linear_out/bias"] += np.concatenate([np.zeros(A), -0.5 * np.ones(A)]).astype(np.float32)
    ctx.params_set(0, O.pack(p, O.gnn_param_shapes(2 * A, layer=layer)))
    return p


class GnnOracleRollout(OracleRollout):
    layer = "mpnn"

    def __init__(self, cfg, inst, params, filt):
        super().__init__(cfg, inst, params[0] if isinstance(params, list) else params, filt)
        self.params = [params] if not isinstance(params, list) else params
        T, N_ = cfg.frag_len, cfg.n_envs
        self.rec[0]["obs"] = np.zeros((T, N_ * 4, 93), np.float32)
        self.node_tables = [inst.obs_indices[a] for a in self.agents]

    def _observe_block(self, obs):
        normed = O.mean_std_filter(obs, self.rs, update=True, clip=self.cfg.filter_clip)
        X = np.stack([O.graph_observation(obs[e].astype(np.float64), normed[e], self.node_tables)
                      for e in range(obs.shape[0])]).astype(np.float32)
        return [X]

    def _forward_all(self):
        X = self.stage[0]
        N_ = X.shape[0]
        Xr = np.repeat(X, 4, axis=0)                     # row c = e * 4 + n
        node = np.tile(np.arange(4), N_)
        logits, value, _ = O.gnn_forward(self.params[0], Xr, node, layer=self.layer)
        return Xr, node, logits, value

    def act(self, t, eps):
        cfg = self.cfg
        A = cfg.act_dim
        Xr, node, logits, value = self._forward_all()
        a = O.dg_sample(logits, eps.reshape(-1, A))
        r = self.rec[0]
        r["obs"][t, :, :92] = Xr.reshape(-1, 92)
        r["obs"][t, :, 92] = node
        r["act"][t], r["logits"][t] = a, logits
        r["logp"][t], r["vf"][t] = O.dg_logp(logits, a), value
        actions = np.zeros((cfg.n_envs, 8), np.float32)
        for s, name in enumerate(self.agents):
            actions[:, self.inst.action_indices[name]] = np.clip(a.reshape(-1, 4, A)[:, s], -1, 1)
        return actions

    def bootstrap(self):
        self.last_v = [self._forward_all()[3]]


def drift_check(got, model, params, shapes, batch, sh, pe, kl, steps, factor=4.0, floor=2e-7, cfg=None):
    """Long-horizon parameter parity against the fp64 trajectory of the same algorithm.

    Runs the oracle's minibatch loop in fp32 (numpy) and in fp64 (oracle.with_dtype) over the
    same schedule; e32 = max |theta_fp32 - theta_fp64| is what fp32 rounding alone costs over
    `steps` dependent steps.  The HIP parameters `got` must satisfy
    max |got - theta_fp64| <= factor * e32 + floor and stay within 1e-5 of the fp32 oracle.
    Returns (e32, egpu, max |got - theta_fp32|, fp64 per-step stats, fp64 params)."""
    O64 = O.with_dtype(np.float64)
    n = sum(int(np.prod(s)) for _, s in shapes)
    cfg = {"entropy_coeff": 0.0, **(cfg or {})}
    new32, _ = O.ppo_update(model, params, shapes, O.Adam(n), batch, sh, pe, np.float32(kl), cfg, steps=steps)
    p64 = {k: np.asarray(v, np.float64) for k, v in params.items()}
    new64, st64 = O64.ppo_update(model, p64, shapes, O64.Adam(n), batch, sh, pe, kl, cfg, steps=steps)
    th32 = O.pack(new32, shapes).astype(np.float64)
    th64 = O64.pack(new64, shapes)
    got = np.asarray(got, np.float64)
    e32, egpu, d32 = np.abs(th32 - th64).max(), np.abs(got - th64).max(), np.abs(got - th32).max()
    moved = np.abs(th64 - O.pack(params, shapes)).max()
    print(f"\n{model} {steps} steps: max |theta moved| {moved:.3g}; max dev from fp64: numpy fp32 {e32:.3g}, "
          f"HIP {egpu:.3g}; max |HIP - numpy fp32| {d32:.3g}")
    assert egpu <= factor * e32 + floor, (egpu, e32)
    assert d32 <= 1e-5, d32
    return e32, egpu, d32, st64, new64


def strict_params_check(got, model, params, shapes, batch, sh, pe, kl, steps, cfg=None, adam=None,
                        lr=3e-4, msg="", safety=4.0, max_exempt_frac=2e-3):
    """Short-horizon parameter parity against the fp64 trajectory.

    Criterion: every parameter of `got` within 1e-5 (absolute) of the fp64 trajectory of the
    same algorithm (oracle.with_dtype(np.float64), same schedule, same starting Adam state),
    except the entries whose fp64 gradient sits below the fp32 noise floor.  Why those: Adam
    scales every entry's step by that entry's own gradient history (on a fresh state the first
    step is lr * sign(g)), so an entry whose gradient is comparable to fp32 rounding gets a step
    whose size -- even whose sign -- the rounding picks.  The floor at step k is
    n_k = max_{i in V} |g32_k,i - g64_k,i| over the entries of the entry's variable V (one
    layer's kernel or bias), the clipped-gradient (Adam input) error of the numpy fp32 run;
    entry i is exempt when  min_k |g64_k,i| <= safety * lr * steps * n_k / 1e-5, i.e. when
    gradient rounding of `safety` x numpy's could move the entry's accumulated Adam steps by
    the 1e-5 bar.  Exempt entries keep the Adam bound |got - fp64| <= 2 lr steps.  The numpy
    fp32 run must meet the same criterion, so the exemption is a property of fp32 arithmetic,
    not of the HIP kernels.  The count of entries that actually use the exemption (beyond 1e-5)
    is printed and bounded by `max_exempt_frac`.  Returns (n_beyond, n_exemptible, n_params)."""
    O64 = O.with_dtype(np.float64)
    n = sum(int(np.prod(s)) for _, s in shapes)
    cfg = {"entropy_coeff": 0.0, **(cfg or {})}

    def adam_for(mod):
        a = mod.Adam(n, lr=lr)
        if adam is not None:
            dt = np.float64 if mod is O64 else np.float32
            a.m, a.v = np.asarray(adam.m, dt).copy(), np.asarray(adam.v, dt).copy()
            a.b1p, a.b2p = mod.F32(adam.b1p), mod.F32(adam.b2p)
        return a

    g32, g64 = [], []
    new32, _ = O.ppo_update(model, params, shapes, adam_for(O), batch, sh, pe, np.float32(kl), cfg,
                            steps=steps, gradlog=g32)
    p64 = {k: np.asarray(v, np.float64) for k, v in params.items()}
    new64, _ = O64.ppo_update(model, p64, shapes, adam_for(O64), batch, sh, pe, kl, cfg, steps=steps,
                              gradlog=g64)
    assert len(g64) == steps, (len(g64), steps)
    th32 = O.pack(new32, shapes).astype(np.float64)
    th64 = O64.pack(new64, shapes)
    got = np.asarray(got, np.float64)
    # the floor per step and per variable (kernel / bias of one layer): rounding scales with
    # the magnitudes summed into that variable's gradient
    sizes = [int(np.prod(s)) for _, s in shapes]
    err = np.abs(np.stack(g32).astype(np.float64) - np.stack(g64))
    floor = np.concatenate([np.repeat(e.max(axis=1, keepdims=True), e.shape[1], axis=1)
                            for e in np.split(err, np.cumsum(sizes)[:-1], axis=1)], axis=1)
    gmin_over_floor = np.min(np.abs(np.stack(g64)) / np.maximum(floor, 1e-30), axis=0)
    exempt = gmin_over_floor <= safety * lr * steps / 1e-5
    dev_hip, dev_np = np.abs(got - th64), np.abs(th32 - th64)
    over = dev_hip > 1e-5
    n_ex, n_over = int(exempt.sum()), int(over.sum())
    print(f"\n{msg} {model} {steps} steps: max dev from fp64 HIP {dev_hip.max():.3g}, numpy fp32 "
          f"{dev_np.max():.3g}; {n_over} of {n} entries beyond 1e-5 (all must be among the {n_ex} whose "
          f"fp64 gradient sits below the fp32 floor)")
    assert np.all(dev_np[~exempt] <= 1e-5), (msg, "numpy fp32 fails its own criterion", dev_np[~exempt].max())
    assert not np.any(over & ~exempt), (msg, "entries beyond 1e-5 with a gradient above the fp32 floor",
                                        np.flatnonzero(over & ~exempt)[:10], dev_hip[over & ~exempt].max())
    assert n_over <= max(1, max_exempt_frac * n), (msg, n_over, n)
    if n_over:
        assert dev_hip.max() <= 2 * lr * steps + 1e-5, (msg, dev_hip.max())
    return n_over, n_ex, n


class HipLockstep:
    """The HIP trajectory of policy `pid`, one step at a time (ddrl_ppo_update_from: bit-identical
    to one uninterrupted launch), with the HIP gradient of a minibatch from its current state
    (ddrl_ppo_grad)."""

    def __init__(self, ctx, pid, theta0, sh, pe, kl):
        import torch
        self.ctx, self.pid, self.kl = ctx, pid, kl
        P = ctx.cfg.n_policies
        self.P = P
        self.dsh = [torch.from_numpy(np.ascontiguousarray(sh)).cuda() if q == pid else None for q in range(P)]
        self.dpe = [torch.from_numpy(np.ascontiguousarray(pe)).cuda() if q == pid else None for q in range(P)]
        n = theta0.size
        self.gbuf = torch.zeros(n, device="cuda")
        self.snaps = {}
        ctx.params_set(pid, theta0)
        ctx.adam_set(pid, np.zeros(n, np.float32), np.zeros(n, np.float32), 0.9, 0.999)

    def grad(self, rows):
        import torch
        r = torch.from_numpy(np.ascontiguousarray(rows)).cuda()
        self.ctx.ppo_grad(self.pid, r, rows.size, self.kl, self.gbuf)
        self.ctx.synchronize()
        return self.gbuf.cpu().numpy().astype(np.float64)

    def step(self, k):
        self.ctx.ppo_update(1 << self.pid, self.dsh, self.dpe, [self.kl] * self.P, max_steps=1, step0=k)

    def theta(self):
        self.ctx.synchronize()
        return self.ctx.params_get(self.pid).astype(np.float64)


class NumpyLockstep:
    """The numpy fp32 oracle's trajectory, one step at a time, with its gradient of a minibatch
    from its current state: an fp32 implementation whose tie outcomes are numpy's."""

    def __init__(self, params, shapes, batch, sh, pe, kl, model="ffn"):
        self.shapes, self.batch, self.sh, self.pe, self.kl, self.model = shapes, batch, sh, pe, kl, model
        self.th = O.pack(params, shapes)
        self.adam = O.Adam(self.th.size)
        self.snaps = {}

    def _fwd_bwd(self, rows):
        b, p = self.batch, O.unpack(self.th, self.shapes)
        if self.model == "gnn":
            logits, value, cache = O.gnn_forward(p, b["X"][rows], b["node_idx"][rows])
        else:
            logits, value, cache = O.ffn_forward(p, b["obs"][rows])
        dl, dv, _ = O.ppo_loss_rows(logits, value, b["actions"][rows], b["logits"][rows], b["logp"][rows],
                                    b["vf_preds"][rows], b["adv"][rows], b["vt"][rows], np.float32(self.kl))
        g = (O.gnn_backward if self.model == "gnn" else O.ffn_backward)(p, cache, dl, dv)
        return [g[nm] for nm, _ in self.shapes]

    def grad(self, rows):
        return np.concatenate([g.reshape(-1) for g in self._fwd_bwd(rows)]).astype(np.float64)

    def step(self, k):
        nb = self.pe.shape[1]
        rows = O.minibatch_rows(self.sh, self.pe, k // nb, k % nb)
        clipped, _ = O.clip_by_global_norm(self._fwd_bwd(rows))
        self.th = self.adam.apply(self.th, np.concatenate([c.reshape(-1) for c in clipped]))

    def theta(self):
        return np.asarray(self.th, np.float64)


def tie_following_trajectory(ctx, pid, params, shapes, batch, sh, pe, kl, steps, horizons, tol=None,
                             max_flips=8, log=None, model="ffn", detect=2e-4, impl=None, pool=48, missed=None):
    """The fp64 trajectory of the minibatch loop that takes an fp32 implementation's outcome at
    every clip decision it took the other way ("Near-ties").

    PPO's loss has two clip decisions per row, each a discontinuity of the gradient: the
    surrogate passes gradient or not (ratio against 1 +- clip) and the value term passes gradient
    or not (|V - vf_old| against vf_clip, and (V - vt)^2 against the clipped square).  When a
    decision's deciding quantity lies within fp32 resolution of its threshold, its outcome is set
    by the implementation's rounding -- TF's, numpy's, the HIP kernel's alike -- and a flip changes
    that step's gradient by a finite amount; the trajectories bifurcate there.

    Lockstep (round 6): the implementation (`impl`: HipLockstep over `ctx` by default, or
    NumpyLockstep) walks its own trajectory one step at a time, and at every step returns its
    gradient of that step's minibatch from its own state.  The fp64 algorithm runs beside it from
    its own state; where the two gradients differ by more than `detect` (relative to the largest
    fp64 entry) the decisions that flipped are found greedily among the `pool` decisions of
    smallest margin (oracle.ppo_branches), each flip kept only if it halves the difference, and
    the fp64 step takes the implementation's outcomes (oracle.ppo_loss_rows(force=...)).  No
    margin tolerance is involved: a flip of any margin within the pool is seen.  A step whose
    difference stays above `detect` after the search is appended to `missed` (step, difference
    before, after) when a list is given.  Everything else is the unmodified fp64 algorithm.
    (`tol` is accepted for the older signature and unused.)

    Returns (snapshots {H: fp64 theta}, per-step fp64 stats, ties) and leaves the implementation's
    own parameters at each horizon in impl.snaps; ties =
    one record per followed decision: (step, kind, row, margin, fp64 outcome, implementation's
    outcome, gradient difference with the implementation's outcome, with fp64's), differences
    relative to max |g_fp64|.  model: "ffn" (batch "obs") or "gnn" (batch "X", "node_idx")."""
    O64 = O.with_dtype(np.float64)
    n = sum(int(np.prod(s_)) for _, s_ in shapes)
    theta0 = O.pack(params, shapes)
    if impl is None:
        impl = HipLockstep(ctx, pid, theta0, sh, pe, kl)
    theta = theta0.astype(np.float64)
    adam = O64.Adam(n)
    epochs, nb = pe.shape
    snaps, stats, ties = {}, [], []
    hset = set(horizons)
    cols = ("actions", "logits", "logp", "vf_preds", "adv", "vt")
    backward = O64.gnn_backward if model == "gnn" else O64.ffn_backward

    def flat(g):
        return np.concatenate([g[nm].reshape(-1) for nm, _ in shapes])

    for k in range(steps):
        rows = O.minibatch_rows(sh, pe, k // nb, k % nb)
        p = O64.unpack(theta, shapes)
        if model == "gnn":
            logits, value, cache = O64.gnn_forward(p, batch["X"][rows], batch["node_idx"][rows])
        else:
            logits, value, cache = O64.ffn_forward(p, batch["obs"][rows])
        args = [batch[c][rows] for c in cols]
        dl, dv, st = O64.ppo_loss_rows(logits, value, *args, np.float64(kl))
        g_nat = flat(backward(p, cache, dl, dv))
        gh = impl.grad(rows)
        scale = max(np.abs(g_nat).max(), 1e-30)
        err_nat = np.abs(gh - g_nat).max() / scale
        if err_nat > detect:
            pol_on, pol_m, vf_on, m_sq, m_in = O.ppo_branches(logits, value, args[0], args[2], args[3], args[4],
                                                              args[5])
            # the value decision's margin: the quantity that decides it (inside the clip: |dv|
            # against vf_clip; outside: the two squares)
            vm = np.where(m_in > 0, m_in, np.minimum(np.abs(m_in), np.abs(m_sq)))
            cand = sorted([(abs(float(pol_m[i])), "pol", int(i), float(pol_m[i]), bool(pol_on[i]))
                           for i in range(rows.size)] +
                          [(abs(float(vm[i])), "vf", int(i), float(vm[i]), bool(vf_on[i]))
                           for i in range(rows.size)])[:pool]
            f = {"pol": {}, "vf": {}}
            cur, chosen = err_nat, {}
            for _ in range(max_flips):
                best = None
                for _, kind, i, m, nat in cand:
                    if i in f[kind]:
                        continue
                    f2 = {"pol": dict(f["pol"]), "vf": dict(f["vf"])}
                    f2[kind][i] = not nat
                    d2, v2, _ = O64.ppo_loss_rows(logits, value, *args, np.float64(kl), force=f2)
                    e2 = np.abs(gh - flat(backward(p, cache, d2, v2))).max() / scale
                    if best is None or e2 < best[0]:
                        best = (e2, kind, i, m, nat)
                if best is None or best[0] > 0.5 * cur:
                    break
                cur = best[0]
                f[best[1]][best[2]] = not best[4]
                chosen[(best[1], best[2])] = (best[3], best[4])
                if cur <= detect:
                    break
            if cur > detect:
                if missed is not None:
                    missed.append((k, float(err_nat), float(cur)))
                if log:
                    log(f"step {k}: gradient difference {err_nat:.3g} ({cur:.3g} after the flips found) not explained")
            if chosen:
                for (kind, i), (m, nat) in chosen.items():
                    # the runner-up: this decision toggled back to fp64's outcome
                    f3 = {"pol": dict(f["pol"]), "vf": dict(f["vf"])}
                    f3[kind][i] = nat
                    d3, v3, _ = O64.ppo_loss_rows(logits, value, *args, np.float64(kl), force=f3)
                    e3 = np.abs(gh - flat(backward(p, cache, d3, v3))).max() / scale
                    ties.append((k, kind, i, m, nat, not nat, cur, e3))
                    if log:
                        log(f"step {k}: {kind} clip of row {i}, fp64 margin {m:.3g}, fp64 {'on' if nat else 'off'}, "
                            f"implementation {'off' if nat else 'on'} (relative gradient difference {cur:.3g}; "
                            f"{e3:.3g} with fp64's outcome)")
                dl, dv, st = O64.ppo_loss_rows(logits, value, *args, np.float64(kl), force=f)
        g = backward(p, cache, dl, dv)
        clipped, gn = O64.clip_by_global_norm([g[nm] for nm, _ in shapes])
        theta = adam.apply(theta, np.concatenate([c.reshape(-1) for c in clipped]))
        st["grad_gnorm"] = float(gn)
        stats.append(st)
        impl.step(k)
        if k + 1 in hset:
            snaps[k + 1] = theta.copy()
            impl.snaps[k + 1] = impl.theta()
    return snaps, stats, ties
