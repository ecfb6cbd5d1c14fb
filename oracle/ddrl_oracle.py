"""CPU oracle for DDRL's rollout + multi-agent PPO hot path (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker or the CPU baseline.  The product path
(ddrl_amd/*, libddrl_hip.so) never calls it.

Pinning status (see DESIGN.md "Oracle"):
  * Layout tables (observation gather, action scatter, contact-force tables) are pinned
    by tests/golden/layout_tables.json.  That file is extracted from the reference's own
    source literals.
  * The PPO loss composition  total = policy_loss + beta*kl + vf_coeff*vf_loss
    - ent_coeff*entropy  is pinned by the known-answer learner stats that the reference
    recorded (tests/golden/learner_stats.json, 75 policy records).
  * Everything else is a restatement of published algorithms.  These live in
    third-party code that is absent from the reference tree: ray[rllib]==1.0.1
    (DiagGaussian, compute_advantages, PPOLoss, clip_gradients, MeanStdFilter /
    RunningStat, TrainTFMultiGPU schedule, update_kl) and tensorflow==2.3.1 (Keras
    Dense, tanh, tf1 AdamOptimizer / ApplyAdam, clip_by_global_norm).  The reference's
    own model code is restated from models/*.py.  No reference test pins their outputs,
    so these parts are "parity unpinned" against RLlib/TF.  Their gradients are
    cross-checked against torch autograd in tests/test_oracle.py.

Precision follows the reference: the NN math is float32 (TF graph dtype), while the
observation filter (RunningStat) and GAE are float64 (numpy defaults in RLlib).
"""
from __future__ import annotations

import math

import numpy as np
from scipy.signal import lfilter

F32 = np.float32
LOG2PI = float(np.log(2.0 * np.pi))


# --------------------------------------------------------------------------------------
# A.1  RunningStat / MeanStdFilter  (ray/rllib/utils/filter.py, ray 1.0.1);
#      env-side singleton: simulation_envs/observation_filter.py:3-12,
#      quantruped_adaptor_multi_environment.py:83-85
# --------------------------------------------------------------------------------------
class RunningStat:
    def __init__(self, shape):
        self.n = 0
        self.M = np.zeros(shape, np.float64)
        self.S = np.zeros(shape, np.float64)

    def push(self, x):
        x = np.asarray(x, np.float64)
        n1 = self.n
        self.n += 1
        if self.n == 1:
            self.M[...] = x
        else:
            delta = x - self.M
            self.M[...] += delta / self.n
            self.S[...] += delta * delta * n1 / self.n

    def update(self, other):  # Chan et al. parallel merge (RunningStat.update)
        n1, n2 = self.n, other.n
        n = n1 + n2
        if n == 0:
            return
        delta = self.M - other.M
        self.M[...] = (n1 * self.M + n2 * other.M) / n
        self.S[...] = self.S + other.S + delta * delta * n1 * n2 / n
        self.n = n

    @property
    def var(self):
        return self.S / (self.n - 1) if self.n > 1 else np.square(self.M)

    @property
    def std(self):
        return np.sqrt(self.var)


def mean_std_filter(x, rs: RunningStat, update=True, clip=10.0):
    """MeanStdFilter.__call__: a batched call pushes every row first, then normalizes
    the whole batch with the final statistics."""
    x = np.asarray(x, np.float64)
    if update:
        if x.ndim == rs.M.ndim + 1:
            for row in x:
                rs.push(row)
        else:
            rs.push(x)
    x = x - rs.M
    x = x / (rs.std + 1e-8)
    if clip:
        x = np.clip(x, -clip, clip)
    return x


# --------------------------------------------------------------------------------------
# a1 / a3 / a7 / a8  env-side routing
# --------------------------------------------------------------------------------------
def distribute_observations(obs_normed, obs_index):
    """quantruped_adaptor_multi_environment.py:124-136: per-agent gather."""
    return {a: obs_normed[..., idx] for a, idx in obs_index.items()}


LEG_ANGLES = (45.0, 135.0, -135.0, -45.0)  # FL, HL, HR, FR


def quaternion_multiply(q1, q2):
    """quantruped_GraphDecentralizedController_environments.py:145-152 (x,y,z,w naming)."""
    x1, y1, z1, w1 = q1
    x2, y2, z2, w2 = q2
    return np.array([
        x1 * w2 + y1 * z2 - z1 * y2 + w1 * x2,
        -x1 * z2 + y1 * w2 + z1 * x2 + w1 * y2,
        x1 * y2 - y1 * x2 + z1 * w2 + w1 * z2,
        -x1 * x2 - y1 * y2 - z1 * z2 + w1 * w2])


def leg_encoding_ego(angle_deg, obs_raw):
    """:154-161  quat_mul(obs[1:5], [0, 0, sin(a/2), cos(a/2)])."""
    rad = np.deg2rad(angle_deg / 2.0)
    return quaternion_multiply(obs_raw[1:5], [0.0, 0.0, np.sin(rad), np.cos(rad)])


def graph_observation(obs_raw, obs_normed, node_index):
    """:218-245  X[n] = concat(z[idx_n], leg_encoding_ego(angle_n, raw obs)) -> [4, 23]."""
    rows = []
    for n, idx in enumerate(node_index):
        rows.append(np.concatenate((obs_normed[idx], leg_encoding_ego(LEG_ANGLES[n], obs_raw))))
    return np.stack(rows)


def ring_adjacency():
    """:167-190  edges FL->HL->HR->FR->FL plus reverses; adj[sender, receiver] = 1."""
    edges = [(0, 1), (1, 2), (2, 3), (3, 0), (1, 0), (2, 1), (3, 2), (0, 3)]
    adj = np.zeros((4, 4))
    for s, r in edges:
        adj[s, r] = 1.0
    return adj


def concatenate_actions(action_dict, action_index):
    """:205-212"""
    out = np.empty(8)
    for a, act in action_dict.items():
        out[action_index[a]] = act
    return out


def per_leg_reward(fw_reward, cfrc_ext, action_dict, contact_tables, ctrl_w, contact_w,
                   norm_reward=False):
    """:160-171 (contact cost per agent) and :188-203 (per-leg reward)."""
    cc = contact_w * np.square(np.clip(cfrc_ext, -1.0, 1.0))
    n = len(action_dict)
    rew = {}
    for a, act in action_dict.items():
        idx, w = contact_tables[a]
        contact = np.sum(cc[idx] * np.asarray(w)[:, None])
        ctrl = ctrl_w * np.sum(np.square(act))
        rew[a] = fw_reward - n * (ctrl + contact) if norm_reward else fw_reward / n - ctrl - contact
    return rew


def tvel_forward_reward(x_velocity, target_velocity):
    """QuAntrupedTVelEnv.compute_forward_reward (simulation_envs/quantruped_v3.py:391-392);
    target_velocity may be per env (an array broadcast against x_velocity)."""
    tv = np.asarray(target_velocity, np.float64)
    return (1.0 + 1.0 / tv) * (1.0 / (np.abs(x_velocity - tv) + 1.0) - 1.0 / (tv + 1.0))


def target_velocity_pmf(target_velocity_list):
    """The distribution of one episode's target velocity: the adaptor draws
    random.choice(target_velocity_list) at construction and on every reset()
    (simulation_envs/quantruped_adaptor_multi_environment.py:47-50, 214-216), and CPython's
    random.choice picks seq[_randbelow(len(seq))] -- every list POSITION equally likely, so a
    value listed twice is drawn twice as often.  Returns {value: probability}."""
    tvs = list(target_velocity_list) if isinstance(target_velocity_list, (list, tuple)) else [target_velocity_list]
    pmf = {}
    for v in tvs:
        pmf[float(v)] = pmf.get(float(v), 0.0) + 1.0 / len(tvs)
    return pmf


def global_reward(fw_reward, cfrc_ext, action_dict, ctrl_w, contact_w):
    """:173-186"""
    contact = contact_w * np.sum(np.square(np.clip(cfrc_ext, -1.0, 1.0)))
    ctrl = sum(np.sum(np.square(a)) for a in action_dict.values())
    n = len(action_dict)
    return {a: (fw_reward - ctrl_w * ctrl - contact) / n for a in action_dict}


# --------------------------------------------------------------------------------------
# a5  GlorotUniformScaled (models/glorot_uniform_scaled_initializer.py:3-19)
# --------------------------------------------------------------------------------------
def glorot_uniform(rng, fan_in, fan_out, scale=1.0):
    limit = math.sqrt(6.0 * scale / (fan_in + fan_out))
    return rng.uniform(-limit, limit, size=(fan_in, fan_out)).astype(F32)


# --------------------------------------------------------------------------------------
# a4  fcnet (models/fcnet_glorot_uniform_init.py:17-125), Keras variable order
# --------------------------------------------------------------------------------------
def ffn_param_shapes(d, num_outputs, hidden=64):
    return [
        ("fc_1/kernel", (d, hidden)), ("fc_1/bias", (hidden,)),
        ("fc_value_1/kernel", (d, hidden)), ("fc_value_1/bias", (hidden,)),
        ("fc_2/kernel", (hidden, hidden)), ("fc_2/bias", (hidden,)),
        ("fc_value_2/kernel", (hidden, hidden)), ("fc_value_2/bias", (hidden,)),
        ("fc_out/kernel", (hidden, num_outputs)), ("fc_out/bias", (num_outputs,)),
        ("value_out/kernel", (hidden, 1)), ("value_out/bias", (1,)),
    ]


def ffn_init(rng, d, num_outputs, hidden=64):
    p = {}
    for name, shape in ffn_param_shapes(d, num_outputs, hidden):
        if name.endswith("bias"):
            p[name] = np.zeros(shape, F32)
        else:
            scale = 0.01 if name.startswith(("fc_out", "value_out")) else 1.0
            p[name] = glorot_uniform(rng, shape[0], shape[1], scale)
    return p


def pack(params, shapes):
    return np.concatenate([params[n].reshape(-1) for n, _ in shapes]).astype(F32)


def unpack(flat, shapes):
    out, o = {}, 0
    for n, s in shapes:
        k = int(np.prod(s))
        out[n] = np.asarray(flat[o:o + k], F32).reshape(s)
        o += k
    return out


def ffn_forward(p, x):
    x = np.asarray(x, F32)
    h1 = np.tanh(x @ p["fc_1/kernel"] + p["fc_1/bias"])
    h2 = np.tanh(h1 @ p["fc_2/kernel"] + p["fc_2/bias"])
    logits = h2 @ p["fc_out/kernel"] + p["fc_out/bias"]
    g1 = np.tanh(x @ p["fc_value_1/kernel"] + p["fc_value_1/bias"])
    g2 = np.tanh(g1 @ p["fc_value_2/kernel"] + p["fc_value_2/bias"])
    value = (g2 @ p["value_out/kernel"] + p["value_out/bias"])[:, 0]
    return logits.astype(F32), value.astype(F32), (x, h1, h2, g1, g2)


def ffn_backward(p, cache, dlogits, dvalue):
    """Manual reverse of a4 (tanh' = 1 - y^2).  Returns grads keyed like params."""
    x, h1, h2, g1, g2 = cache
    g = {}
    dlogits = np.asarray(dlogits, F32)
    g["fc_out/kernel"] = h2.T @ dlogits
    g["fc_out/bias"] = dlogits.sum(0)
    dz2 = (dlogits @ p["fc_out/kernel"].T) * (1 - h2 * h2)
    g["fc_2/kernel"] = h1.T @ dz2
    g["fc_2/bias"] = dz2.sum(0)
    dz1 = (dz2 @ p["fc_2/kernel"].T) * (1 - h1 * h1)
    g["fc_1/kernel"] = x.T @ dz1
    g["fc_1/bias"] = dz1.sum(0)
    dv = np.asarray(dvalue, F32)[:, None]
    g["value_out/kernel"] = g2.T @ dv
    g["value_out/bias"] = dv.sum(0)
    dy2 = (dv @ p["value_out/kernel"].T) * (1 - g2 * g2)
    g["fc_value_2/kernel"] = g1.T @ dy2
    g["fc_value_2/bias"] = dy2.sum(0)
    dy1 = (dy2 @ p["fc_value_2/kernel"].T) * (1 - g1 * g1)
    g["fc_value_1/kernel"] = x.T @ dy1
    g["fc_value_1/bias"] = dy1.sum(0)
    return {k: v.astype(F32) for k, v in g.items()}


# --------------------------------------------------------------------------------------
# f4  "cup": fcnet + trainable leg coupling (models/coupling_net_glorot_uniform_init.py:11-30,
#     model :32-137; registered models/__init__.py:10).  LegCoupling.build starts the table
#     at [[1,1],[-1,-1],[-1,-1],[1,1]] (:20); call() pads it with ones for the log-std half
#     (:27) and gathers the row of the agent's leg index (:28), so only the means are scaled.
#     The variable follows the fcnet variables (register_variables order, :136-137).
# --------------------------------------------------------------------------------------
LEG_COUPLING_INIT = np.array([[1, 1], [-1, -1], [-1, -1], [1, 1]], F32)


def cup_param_shapes(d, A, hidden=64):
    return ffn_param_shapes(d, 2 * A, hidden) + [("leg_coupling", (4, A))]


def cup_init(rng, d, A, hidden=64):
    p = ffn_init(rng, d, 2 * A, hidden)
    p["leg_coupling"] = np.resize(LEG_COUPLING_INIT, (4, A)).astype(F32)
    return p


def cup_forward(p, x, leg):
    logits, value, cache = ffn_forward(p, x)
    leg = np.asarray(leg).reshape(-1).astype(np.int64)
    A = p["leg_coupling"].shape[1]
    coef = np.concatenate([p["leg_coupling"], np.ones_like(p["leg_coupling"])], 1)[leg]
    return (logits * coef).astype(F32), value, (cache, logits, leg, coef, A)


def cup_backward(p, cache, dlogits, dvalue):
    fcache, pre, leg, coef, A = cache
    dlogits = np.asarray(dlogits, F32)
    g = ffn_backward(p, fcache, dlogits * coef, dvalue)
    gc = np.zeros((4, A), F32)
    np.add.at(gc, leg, (dlogits * pre)[:, :A])
    g["leg_coupling"] = gc
    return g


# --------------------------------------------------------------------------------------
# a9 / a10  GraphNet + MPNN (models/graph_net.py:8-45, models/gcn.py:39-94,
#           models/shared_graphnet_glorot_uniform_init.py:14-58); f4 alternates GCN / MPNN2 /
#           GAT1 (models/gcn.py:7-37, 96-150, 153-206; models/graph_ops.py:3-26)
# --------------------------------------------------------------------------------------
# The message-passing layer of GraphNet is MPNN in the reference (graph_net.py:20); GCN, MPNN2
# and GAT1 (gcn.py:7-37, 96-150, 153-206, with graph_ops.py:13-26) are the alternates that line
# selects.  All four take (x [B, n, 64], adj [B, n, n]) and return tanh(...) [B, n, 64] with
# no bias (use_bias=False, graph_net.py:22).  Edges are tf.where(adj): (batch, sender = row,
# receiver = column).
GNN_LAYERS = ("mpnn", "gcn", "mpnn2", "gat1")


def gnn_layer_shapes(layer, hidden=64):
    return {"mpnn": [("mpnn/msg_transform/kernel", (hidden, hidden)), ("mpnn/node_update/kernel", (hidden, hidden))],
            "gcn": [("gcn/linear/kernel", (hidden, hidden))],
            "mpnn2": [("mpnn2/msg_transform/kernel", (2 * hidden, hidden)), ("mpnn2/node_update/kernel", (2 * hidden, hidden))],
            "gat1": [("gat1/pre_att_linear/kernel", (hidden, hidden)), ("gat1/att_linear/kernel", (2 * hidden, 1))]}[layer]


def gnn_net_shapes(num_outputs, hidden=64, feat=19, qdim=4, layer="mpnn"):
    return ([("state_enc/kernel", (qdim, feat * hidden)), ("state_enc/bias", (feat * hidden,))] +
            gnn_layer_shapes(layer, hidden) +
            [("linear_out/kernel", (hidden, num_outputs)), ("linear_out/bias", (num_outputs,))])


def gnn_param_shapes(num_outputs, hidden=64, layer="mpnn"):
    return ([("actor/" + n, s) for n, s in gnn_net_shapes(num_outputs, hidden, layer=layer)] +
            [("critic/" + n, s) for n, s in gnn_net_shapes(1, hidden, layer=layer)])


def gnn_init(rng, num_outputs, hidden=64, layer="mpnn"):
    """GlorotUniformScaled(1.0) for the encoder and the layer kernels (GAT1 takes Keras'
    default glorot_uniform: the same law), 0.01 for linear_out, zero biases; one draw per
    kernel in variable order."""
    p = {}
    for name, shape in gnn_param_shapes(num_outputs, hidden, layer):
        if name.endswith("bias"):
            p[name] = np.zeros(shape, F32)
        else:
            scale = 0.01 if "linear_out" in name else 1.0
            p[name] = glorot_uniform(rng, shape[0], shape[1], scale)
    return p


def _edges(adj):
    e = (adj != 0).astype(F32)          # e[b, s, r]: edge sender s -> receiver r
    cnt = e.sum(1)                      # in-degree of every receiver
    return e, cnt


def _seg_mean(e, cnt, msg_sr):
    """unsorted_segment_mean over receivers of per-edge messages msg_sr [B, s, r, k]."""
    m = np.einsum("bsr,bsrj->brj", e, msg_sr)
    return np.where(cnt[..., None] > 0, m / np.maximum(cnt[..., None], 1), 0.0).astype(F32)


def _layer_forward(p, pre, layer, h, adj):
    """The message-passing layer; returns y and its cache."""
    if layer == "mpnn":             # gcn.py:57-94
        e, cnt = _edges(adj)
        msg = h @ p[pre + "mpnn/msg_transform/kernel"]
        m = np.einsum("bsr,bsj->brj", e, msg)
        m = np.where(cnt[..., None] > 0, m / np.maximum(cnt[..., None], 1), 0.0).astype(F32)
        y = np.tanh(h @ p[pre + "mpnn/node_update/kernel"] + m)
        return y, (e, cnt)
    if layer == "gcn":              # gcn.py:29-37 with graph_ops.adj_norm (:13-21): D^-1 A
        an = (adj / adj.sum(-1, keepdims=True)).astype(F32)
        hbar = an @ h
        y = np.tanh(hbar @ p[pre + "gcn/linear/kernel"])
        return y, (an, hbar)
    if layer == "mpnn2":            # gcn.py:113-150: message W [x_snd | x_rec], update W [x | m]
        e, cnt = _edges(adj)
        n = h.shape[1]
        hs = np.broadcast_to(h[:, :, None, :], (h.shape[0], n, n, h.shape[2]))   # sender s
        hr = np.broadcast_to(h[:, None, :, :], (h.shape[0], n, n, h.shape[2]))   # receiver r
        cat = np.concatenate([hs, hr], -1)
        esr = cat @ p[pre + "mpnn2/msg_transform/kernel"]
        m = _seg_mean(e, cnt, esr)
        y = np.tanh(np.concatenate([h, m], -1) @ p[pre + "mpnn2/node_update/kernel"])
        return y, (e, cnt, cat, m)
    if layer == "gat1":             # gcn.py:171-206 with graph_ops.segment_softmax (:23-26)
        n = h.shape[1]
        adj1 = np.minimum(F32(1), adj + np.eye(n, dtype=F32)[None])
        e = (adj1 != 0).astype(F32)
        z = h @ p[pre + "gat1/pre_att_linear/kernel"]
        a = p[pre + "gat1/att_linear/kernel"][:, 0]
        H = z.shape[2]
        pre_sr = (z @ a[:H])[:, :, None] + (z @ a[H:])[:, None, :]     # concat(z_s, z_r) . a
        lr = np.where(pre_sr > 0, pre_sr, F32(0.2) * pre_sr)           # tf.nn.leaky_relu (0.2)
        ex = np.exp(lr) * e
        S = ex.sum(1)                                                   # per receiver r
        att = (ex / S[:, None, :]).astype(F32)                          # scatter_nd -> [b, s, r]
        y = np.tanh(att @ z)                                            # x'_s = sum_r att[s, r] z_r
        return y, (e, z, a, pre_sr, att)
    raise ValueError(f"unknown gnn layer {layer!r}")


def _layer_backward(p, pre, layer, h, y, cache, dy, g):
    """Gradient of the layer's kernels into g; returns dL/dh."""
    du = dy * (1 - y * y)
    if layer == "mpnn":
        e, cnt = cache
        g[pre + "mpnn/node_update/kernel"] = np.einsum("bnj,bnk->jk", h, du)
        dh = du @ p[pre + "mpnn/node_update/kernel"].T
        dm = np.where(cnt[..., None] > 0, du / np.maximum(cnt[..., None], 1), 0.0)
        dmsg = np.einsum("bsr,brj->bsj", e, dm)
        g[pre + "mpnn/msg_transform/kernel"] = np.einsum("bnj,bnk->jk", h, dmsg)
        return dh + dmsg @ p[pre + "mpnn/msg_transform/kernel"].T
    if layer == "gcn":
        an, hbar = cache
        g[pre + "gcn/linear/kernel"] = np.einsum("bnj,bnk->jk", hbar, du)
        dhbar = du @ p[pre + "gcn/linear/kernel"].T
        return np.einsum("bsn,bsj->bnj", an, dhbar)
    if layer == "mpnn2":
        e, cnt, cat, m = cache
        H = h.shape[2]
        W = p[pre + "mpnn2/node_update/kernel"]
        g[pre + "mpnn2/node_update/kernel"] = np.einsum("bnj,bnk->jk", np.concatenate([h, m], -1), du)
        dcat = du @ W.T
        dh, dm = dcat[..., :H], dcat[..., H:]
        dm = np.where(cnt[..., None] > 0, dm / np.maximum(cnt[..., None], 1), 0.0)
        de = e[..., None] * dm[:, None, :, :]                          # [b, s, r, k]
        Wm = p[pre + "mpnn2/msg_transform/kernel"]
        g[pre + "mpnn2/msg_transform/kernel"] = np.einsum("bsrj,bsrk->jk", cat, de)
        dcat_e = de @ Wm.T
        return dh + dcat_e[..., :H].sum(2) + dcat_e[..., H:].sum(1)
    if layer == "gat1":
        e, z, a, pre_sr, att = cache
        H = z.shape[2]
        datt = np.einsum("bsj,brj->bsr", du, z) * e
        dz = np.einsum("bsr,bsj->brj", att, du)
        colsum = (att * datt).sum(1)                                     # per receiver r
        dex = att * (datt - colsum[:, None, :])                          # softmax over senders of r
        dpre = dex * np.where(pre_sr > 0, F32(1), F32(0.2))
        dps, dur = dpre.sum(2), dpre.sum(1)                              # d(z_s.a1), d(z_r.a2)
        g[pre + "gat1/att_linear/kernel"] = np.concatenate(
            [np.einsum("bs,bsj->j", dps, z), np.einsum("br,brj->j", dur, z)])[:, None]
        dz = dz + dps[..., None] * a[:H] + dur[..., None] * a[H:]
        g[pre + "gat1/pre_att_linear/kernel"] = np.einsum("bnj,bnk->jk", h, dz)
        return dz @ p[pre + "gat1/pre_att_linear/kernel"].T
    raise ValueError(f"unknown gnn layer {layer!r}")


def _graphnet_forward(p, pre, X, node_idx, adj, hidden=64, layer="mpnn"):
    B = X.shape[0]
    f, q = X[..., :-4], X[..., -4:]
    feat = f.shape[-1]
    wn = np.tanh(q @ p[pre + "state_enc/kernel"] + p[pre + "state_enc/bias"])
    wn = wn.reshape(B, 4, feat, hidden)
    h = np.tanh(np.einsum("bni,bnij->bnj", f, wn))
    y, lc = _layer_forward(p, pre, layer, h, adj)
    ysel = y[np.arange(B), node_idx]
    out = ysel @ p[pre + "linear_out/kernel"] + p[pre + "linear_out/bias"]
    return out.astype(F32), (f, q, wn, h, y, ysel, lc, layer)


def _graphnet_backward(p, pre, cache, dout, node_idx, adj, g):
    f, q, wn, h, y, ysel, lc, layer = cache
    B = f.shape[0]
    g[pre + "linear_out/kernel"] = ysel.T @ dout
    g[pre + "linear_out/bias"] = dout.sum(0)
    dy = np.zeros_like(y)
    dy[np.arange(B), node_idx] = dout @ p[pre + "linear_out/kernel"].T
    dh = _layer_backward(p, pre, layer, h, y, lc, dy, g)
    dz = dh * (1 - h * h)
    dwn = np.einsum("bni,bnj->bnij", f, dz)
    dpre = (dwn * (1 - wn * wn)).reshape(B, 4, -1)
    g[pre + "state_enc/kernel"] = np.einsum("bnc,bnk->ck", q, dpre)
    g[pre + "state_enc/bias"] = dpre.sum((0, 1))


def gnn_forward(p, X, node_idx, adj=None, layer="mpnn"):
    X = np.asarray(X, F32)
    node_idx = np.asarray(node_idx).reshape(-1).astype(np.int64)
    if adj is None:
        adj = np.broadcast_to(ring_adjacency(), (X.shape[0], 4, 4))
    adj = np.asarray(adj, F32)
    logits, ca = _graphnet_forward(p, "actor/", X, node_idx, adj, layer=layer)
    value, cc = _graphnet_forward(p, "critic/", X, node_idx, adj, layer=layer)
    return logits, value[:, 0], (ca, cc, node_idx, adj)


def gnn_backward(p, cache, dlogits, dvalue):
    ca, cc, node_idx, adj = cache
    g = {}
    _graphnet_backward(p, "actor/", ca, np.asarray(dlogits, F32), node_idx, adj, g)
    _graphnet_backward(p, "critic/", cc, np.asarray(dvalue, F32)[:, None], node_idx, adj, g)
    return {k: v.astype(F32) for k, v in g.items()}


# --------------------------------------------------------------------------------------
# a6  DiagGaussian (rllib/models/tf/tf_action_dist.py, ray 1.0.1)
# --------------------------------------------------------------------------------------
def dg_split(logits):
    A = logits.shape[-1] // 2
    return logits[..., :A], logits[..., A:]


def dg_logp(logits, a):
    mean, log_std = dg_split(logits)
    std = np.exp(log_std)
    A = mean.shape[-1]
    return (-0.5 * np.sum(np.square((a - mean) / std), -1) - 0.5 * LOG2PI * A
            - np.sum(log_std, -1)).astype(F32)


def dg_kl(old_logits, new_logits):
    m0, s0 = dg_split(old_logits)
    m1, s1 = dg_split(new_logits)
    return np.sum(s1 - s0 + (np.square(np.exp(s0)) + np.square(m0 - m1)) /
                  (2.0 * np.square(np.exp(s1))) - 0.5, -1).astype(F32)


def dg_entropy(logits):
    _, s = dg_split(logits)
    return np.sum(s + 0.5 * np.log(2.0 * np.pi * np.e), -1).astype(F32)


def dg_sample(logits, eps):
    mean, log_std = dg_split(logits)
    return (mean + np.exp(log_std) * eps).astype(F32)


# --------------------------------------------------------------------------------------
# a11 / a12  GAE (rllib/evaluation/postprocessing.py compute_advantages, ray 1.0.1)
# --------------------------------------------------------------------------------------
def discount(x, gamma):
    return lfilter([1], [1, -gamma], x[::-1], axis=0)[::-1]


def compute_gae(rewards, vf_preds, last_r, gamma=0.99, lambda_=0.95):
    """One trajectory segment.  float64 arithmetic, float32 outputs."""
    vpred_t = np.concatenate([np.asarray(vf_preds, np.float64), [float(last_r)]])
    delta_t = np.asarray(rewards, np.float64) + gamma * vpred_t[1:] - vpred_t[:-1]
    adv = discount(delta_t, gamma * lambda_)
    vt = (adv + np.asarray(vf_preds, np.float32)).astype(np.float32)
    return adv.astype(np.float32), vt


def gae_fragment(rewards, vf_preds, dones, last_v, gamma=0.99, lambda_=0.95):
    """Time-major fragment [T, C] for C independent chains.  The fragment is split into
    episode segments at done flags (postprocess_ppo_gae runs per segment): last_r = 0
    after a done, else V(s_T) = last_v for the trailing segment."""
    T, C = rewards.shape
    adv = np.zeros((T, C), np.float32)
    vt = np.zeros((T, C), np.float32)
    for c in range(C):
        start = 0
        for t in range(T):
            if dones[t, c] or t == T - 1:
                lr = 0.0 if dones[t, c] else last_v[c]
                a, v = compute_gae(rewards[start:t + 1, c], vf_preds[start:t + 1, c], lr,
                                   gamma, lambda_)
                adv[start:t + 1, c] = a
                vt[start:t + 1, c] = v
                start = t + 1
    return adv, vt


def standardize(x):
    """StandardizeFields: (x - mean) / max(1e-4, std), population std.  Statistics are
    accumulated in float64 and applied in float32."""
    x = np.asarray(x, np.float32)
    mean = np.float32(np.mean(x, dtype=np.float64))
    std = np.float32(np.std(x, dtype=np.float64))
    return ((x - mean) / np.maximum(np.float32(1e-4), std)).astype(np.float32), mean, std


# --------------------------------------------------------------------------------------
# a13 / a14  PPOLoss (rllib/agents/ppo/ppo_tf_policy.py, ray 1.0.1) and its gradient
# --------------------------------------------------------------------------------------
def ppo_loss_rows(logits, value, actions, old_logits, old_logp, vf_preds, adv, vt,
                  kl_coeff, clip_param=0.2, vf_clip_param=10.0, vf_loss_coeff=0.5,
                  entropy_coeff=0.0, vf_clip_mode="ray10", force=None):
    """Per-row loss terms and analytic dL/dlogits, dL/dvalue for L = mean over rows.
    The tie rules follow TF's gradient kernels: tf.minimum routes to x where x <= y,
    tf.maximum to x where x >= y, clip_by_value passes for lo <= t <= hi.

    `force` (test infrastructure, the tie-following trajectory of DESIGN.md section 4): an
    optional dict {"pol": {row: bool}, "vf": {row: bool}} that overrides whether a row's
    surrogate / value term passes gradient -- the two clip decisions, whose outcome at a
    near-tie (margin below fp32 resolution) depends on the implementation's rounding."""
    f = F32
    logits = np.asarray(logits, f)
    n, A2 = logits.shape
    A = A2 // 2
    mean, log_std = logits[:, :A], logits[:, A:]
    std = np.exp(log_std)
    om, os_ = old_logits[:, :A], old_logits[:, A:]
    z = (actions - mean) / std
    logp = -0.5 * np.sum(z * z, 1) - f(0.5 * LOG2PI * A) - np.sum(log_std, 1)
    ratio = np.exp(logp - old_logp)
    lo, hi = f(1 - clip_param), f(1 + clip_param)
    cr = np.clip(ratio, lo, hi)
    s1, s2 = adv * ratio, adv * cr
    surr = np.minimum(s1, s2)
    d_ratio = np.where(s1 <= s2, adv, adv * ((ratio >= lo) & (ratio <= hi)))  # d surr
    if force and force.get("pol"):
        for i, on in force["pol"].items():
            d_ratio[i] = adv[i] if on else 0.0
    var1 = np.square(np.exp(os_))
    kl = np.sum(log_std - os_ + (var1 + np.square(om - mean)) / (2 * std * std) - 0.5, 1)
    ent = np.sum(log_std + f(0.5 * np.log(2 * np.pi * np.e)), 1)
    if vf_clip_mode == "ray10":
        vf1 = np.square(value - vt)
        dv = value - vf_preds
        vclip = vf_preds + np.clip(dv, -vf_clip_param, vf_clip_param)
        vf2 = np.square(vclip - vt)
        vf = np.maximum(vf1, vf2)
        d_vf = np.where(vf1 >= vf2, 2 * (value - vt),
                        2 * (vclip - vt) * ((dv >= -vf_clip_param) & (dv <= vf_clip_param)))
        if force and force.get("vf"):
            for i, on in force["vf"].items():
                d_vf[i] = (2 * (value[i] - vt[i]) if vf1[i] >= vf2[i] else 2 * (vclip[i] - vt[i])) if on else 0.0
    else:  # later RLlib: clip((V - VT)^2, 0, vf_clip)
        sq = np.square(value - vt)
        vf = np.clip(sq, 0, vf_clip_param)
        d_vf = 2 * (value - vt) * (sq <= vf_clip_param)
    total = -surr + kl_coeff * kl + vf_loss_coeff * vf - entropy_coeff * ent
    inv_n = f(1.0 / n)
    # dL/dlogp = -d_ratio * ratio ; dlogp/dmean = z/std ; dlogp/dlog_std = z^2 - 1
    g_logp = (-d_ratio * ratio)[:, None]
    d_mean = g_logp * (z / std) + kl_coeff * ((mean - om) / (std * std))
    d_lstd = g_logp * (z * z - 1) + kl_coeff * (1 - (var1 + np.square(om - mean)) / (std * std)) \
        - entropy_coeff
    dlogits = np.concatenate([d_mean, d_lstd], 1) * inv_n
    dvalue = vf_loss_coeff * d_vf * inv_n
    stats = dict(total_loss=np.mean(total), policy_loss=np.mean(-surr), vf_loss=np.mean(vf),
                 kl=np.mean(kl), entropy=np.mean(ent),
                 vf_explained_var=explained_variance(vt, value))
    return dlogits.astype(f), dvalue.astype(f), stats


def ppo_branches(logits, value, actions, old_logp, vf_preds, adv, vt, clip_param=0.2, vf_clip_param=10.0):
    """Test infrastructure: each row's two clip decisions of ppo_loss_rows (ray10 value clip)
    and their relative margins.  pol_on: the surrogate passes gradient (adv > 0: ratio <= 1 +
    clip; adv < 0: ratio >= 1 - clip); vf_on: the value term passes gradient (vf1 >= vf2 or
    |V - vf_old| <= vf_clip).  A margin is the signed relative distance of the deciding quantity
    from its threshold; a decision is ambiguous in fp32 when its margin is within rounding."""
    logits = np.asarray(logits, np.float64)
    A = logits.shape[1] // 2
    mean, log_std = logits[:, :A], logits[:, A:]
    z = (np.asarray(actions, np.float64) - mean) / np.exp(log_std)
    logp = -0.5 * np.sum(z * z, 1) - 0.5 * LOG2PI * A - np.sum(log_std, 1)
    ratio = np.exp(logp - np.asarray(old_logp, np.float64))
    adv = np.asarray(adv, np.float64)
    lo, hi = 1.0 - clip_param, 1.0 + clip_param
    pol_on = np.where(adv > 0, ratio <= hi, np.where(adv < 0, ratio >= lo, True))
    pol_m = np.where(adv > 0, (hi - ratio) / hi, np.where(adv < 0, (ratio - lo) / lo, np.inf))
    value = np.asarray(value, np.float64)
    vf_preds, vt = np.asarray(vf_preds, np.float64), np.asarray(vt, np.float64)
    dv = value - vf_preds
    vcl = vf_preds + np.clip(dv, -vf_clip_param, vf_clip_param)
    vf1, vf2 = (value - vt) ** 2, (vcl - vt) ** 2
    m_sq = (vf1 - vf2) / np.maximum(np.maximum(vf1, vf2), 1e-30)     # > 0: vf1 wins
    m_in = (vf_clip_param - np.abs(dv)) / vf_clip_param                # > 0: inside the clip
    vf_on = (vf1 >= vf2) | (np.abs(dv) <= vf_clip_param)
    return pol_on, pol_m, vf_on, m_sq, m_in


def explained_variance(y, pred):
    """rllib.utils.tf_ops.explained_variance: max(-1, 1 - var(y - pred) / var(y))."""
    vy = np.var(y)
    return float(max(-1.0, 1.0 - np.var(y - pred) / vy)) if vy > 0 else float("nan")


# --------------------------------------------------------------------------------------
# a15 / a16  clip_by_global_norm and tf1 Adam (training_ops ApplyAdam)
# --------------------------------------------------------------------------------------
def clip_by_global_norm(grads, clip_norm=0.5):
    gn = F32(np.sqrt(np.sum([np.sum(np.square(g, dtype=F32)) for g in grads], dtype=F32)))
    scale = F32(clip_norm) * min(F32(1.0) / gn if gn > 0 else F32(np.inf), F32(1.0) / F32(clip_norm))
    return [(g * scale).astype(F32) for g in grads], gn


class Adam:
    """tf1 AdamOptimizer: beta powers are fp32 variables, multiplied after each step."""

    def __init__(self, n, lr=3e-4, b1=0.9, b2=0.999, eps=1e-8):
        self.m = np.zeros(n, F32)
        self.v = np.zeros(n, F32)
        self.lr, self.b1, self.b2, self.eps = F32(lr), F32(b1), F32(b2), F32(eps)
        self.b1p, self.b2p = F32(b1), F32(b2)

    def apply(self, theta, g):
        one = F32(1.0)
        alpha = self.lr * np.sqrt(one - self.b2p) / (one - self.b1p)
        self.m = self.m + (g - self.m) * (one - self.b1)
        self.v = self.v + (g * g - self.v) * (one - self.b2)
        theta = theta - (self.m * alpha) / (np.sqrt(self.v) + self.eps)
        self.b1p = F32(self.b1p * self.b1)
        self.b2p = F32(self.b2p * self.b2)
        return theta.astype(F32)


# --------------------------------------------------------------------------------------
# a17 / a18  minibatch SGD schedule (TrainTFMultiGPU) and KL update
# --------------------------------------------------------------------------------------
def sgd_schedule(rng, n_rows, minibatch=128, epochs=10):
    """Returns (shuffle[n_rows], perms[epochs, nb]) as RLlib draws them: one
    SampleBatch.shuffle() per load, then one permutation of minibatch slots per epoch."""
    shuffle = rng.permutation(n_rows).astype(np.int32)
    nb = max(1, n_rows // minibatch)
    perms = np.stack([rng.permutation(nb) for _ in range(epochs)]).astype(np.int32)
    return shuffle, perms


def minibatch_rows(shuffle, perms, epoch, b, minibatch=128):
    s = int(perms[epoch, b]) * minibatch
    return shuffle[s:s + minibatch]


def update_kl(kl_coeff, sampled_kl, kl_target=0.01):
    if sampled_kl > 2.0 * kl_target:
        kl_coeff *= 1.5
    elif sampled_kl < 0.5 * kl_target:
        kl_coeff *= 0.5
    return kl_coeff


def ppo_update(model, params, shapes, adam, batch, shuffle, perms, kl_coeff, cfg, steps=None, snapshots=None,
               gradlog=None):
    """Runs the minibatch loop for one policy.  `model` is "ffn", "cup" or "gnn".  `batch` is
    a dict of row arrays: obs (+ leg for "cup"; X/node_idx for "gnn"), actions, logits, logp, vf_preds, adv
    (already standardized) and vt.  Returns (params, per-step stats list).  `snapshots`: an
    optional dict {step count: None} filled with the flat parameters after that many steps;
    `gradlog`: an optional list that receives each step's clipped flat gradient (Adam's input)."""
    mb = cfg.get("sgd_minibatch_size", 128)
    epochs, nb = perms.shape
    theta = pack(params, shapes)
    out_stats = []
    k = 0
    for e in range(epochs):
        for b in range(nb):
            if steps is not None and k >= steps:
                return unpack(theta, shapes), out_stats
            rows = minibatch_rows(shuffle, perms, e, b, mb)
            p = unpack(theta, shapes)
            if model == "ffn":
                logits, value, cache = ffn_forward(p, batch["obs"][rows])
            elif model == "cup":
                logits, value, cache = cup_forward(p, batch["obs"][rows], batch["leg"][rows])
            else:
                logits, value, cache = gnn_forward(p, batch["X"][rows], batch["node_idx"][rows],
                                                   layer=cfg.get("gnn_layer", "mpnn"))
            dlogits, dvalue, st = ppo_loss_rows(
                logits, value, batch["actions"][rows], batch["logits"][rows],
                batch["logp"][rows], batch["vf_preds"][rows], batch["adv"][rows],
                batch["vt"][rows], F32(kl_coeff), cfg.get("clip_param", 0.2),
                cfg.get("vf_clip_param", 10.0), cfg.get("vf_loss_coeff", 0.5),
                cfg.get("entropy_coeff", 0.0))
            g = {"ffn": ffn_backward, "cup": cup_backward, "gnn": gnn_backward}[model](p, cache, dlogits, dvalue)
            glist = [g[n] for n, _ in shapes]
            clipped, gn = clip_by_global_norm(glist, cfg.get("grad_clip", 0.5))
            flat = np.concatenate([c.reshape(-1) for c in clipped])
            if gradlog is not None:
                gradlog.append(flat.copy())
            theta = adam.apply(theta, flat)
            st["grad_gnorm"] = float(gn)
            out_stats.append(st)
            k += 1
            if snapshots is not None and k in snapshots:
                snapshots[k] = theta.copy()
    return unpack(theta, shapes), out_stats


def with_dtype(dtype):
    """A private copy of this module whose network arithmetic (forward, loss, backward, clip,
    Adam, the minibatch loop) runs in `dtype` -- np.float64 gives the fp64 trajectory the
    long-horizon parity tests measure fp32 rounding drift against.  Data preprocessing (GAE,
    standardization, the filter) keeps its own fixed precisions."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(f"{__name__}_{np.dtype(dtype).name}", __file__)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.F32 = np.dtype(dtype).type
    return mod
