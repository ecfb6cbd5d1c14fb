"""Pin the CPU oracle: golden fixtures from the reference + torch-autograd cross-checks."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import ddrl_oracle as O
from ddrl_amd.simulation_envs import layouts as L

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_layout_tables_match_reference_literals():
    g = json.load(open(os.path.join(GOLDEN, "layout_tables.json")))
    assert g["OBS_FIELDS"] == L.OBS_FIELDS
    assert g["ACTION_FIELDS"] == L.ACTION_FIELDS
    assert g["CONTACT_FORCE_FIELDS"] == L.CONTACT_FORCE_FIELDS
    assert g["TVEL_OBS_FIELDS"] == L.TVEL_OBS_FIELDS
    n = 0
    for cls, info in g["classes"].items():
        for tab, entries in info.get("tables", {}).items():
            for agent, e in entries.items():
                if tab == "obs_indices":
                    assert L.get_obs_indices(e["prefixes"]) == e["indices"], (cls, agent)
                elif tab == "action_indices":
                    assert L.get_action_indices(e["prefixes"]) == e["indices"], (cls, agent)
                else:
                    idx, w = L.get_contact_force_indices(e["prefixes"], e["weights_in"])
                    assert idx == e["indices"] and w == e["weights"], (cls, agent)
                n += 1
    assert n >= 60


def test_body_first_local_tables():
    # real order is body-first, not the reference's inline comments.
    fl = L.get_obs_indices(['body', 'fl'])
    assert fl == [0, 1, 2, 3, 4, 13, 14, 15, 16, 17, 18, 5, 6, 19, 20, 27, 28, 37, 38]
    assert len(L.get_obs_indices(['body', 'fl', 'hl', 'fr'])) == 35


def test_loss_identity_known_answers():
    """Recorded RLlib learner stats satisfy total = pl + beta*kl + 0.5*vf - c*H."""
    rows = [r for r in json.load(open(os.path.join(GOLDEN, "learner_stats.json")))
            if "total_loss" in r]
    assert len(rows) >= 50
    for r in rows:
        beta = np.float32(r["cur_kl_coeff"])
        tot = (np.float32(r["policy_loss"]) + beta * np.float32(r["kl"]) +
               np.float32(0.5) * np.float32(r["vf_loss"]) -
               np.float32(r["entropy_coeff"]) * np.float32(r["entropy"]))
        assert abs(tot - r["total_loss"]) <= 1e-5 * max(1.0, abs(r["total_loss"])), r
    # the KL schedule: beta in {0.2 * 1.5^i * 0.5^j} in fp32
    betas = {round(r["cur_kl_coeff"], 6) for r in rows}
    allowed = {round(float(np.float32(0.2 * 1.5 ** i * 0.5 ** j)), 6)
               for i in range(40) for j in range(40)}
    assert betas <= allowed


def test_params_fixture():
    p = json.load(open(os.path.join(GOLDEN, "ppo_params_local.json")))
    assert p["gamma"] == 0.99 and p["lambda"] == 0.95 and p["clip_param"] == 0.2
    assert p["vf_clip_param"] == 10.0 and p["grad_clip"] == 0.5 and p["lr"] == 3e-4
    assert p["sgd_minibatch_size"] == 128 and p["num_sgd_iter"] == 10
    assert p["train_batch_size"] == 16000 and p["rollout_fragment_length"] == 200
    assert p["kl_coeff"] == 0.2 and p["kl_target"] == 0.01 and p["shuffle_sequences"]


def test_running_stat_merge_equals_sequential():
    rng = np.random.default_rng(0)
    x = rng.normal(size=(257, 43)) * 3 + 1
    a = O.RunningStat((43,))
    for r in x:
        a.push(r)
    b, c = O.RunningStat((43,)), O.RunningStat((43,))
    for r in x[:100]:
        b.push(r)
    for r in x[100:]:
        c.push(r)
    b.update(c)
    np.testing.assert_allclose(a.M, b.M, rtol=1e-12)
    np.testing.assert_allclose(a.S, b.S, rtol=1e-10)
    assert a.n == b.n == 257


def _torch_ffn_loss(p, batch, beta, cfg):
    t = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in p.items()}
    x = torch.tensor(batch["obs"], dtype=torch.float64)
    h1 = torch.tanh(x @ t["fc_1/kernel"] + t["fc_1/bias"])
    h2 = torch.tanh(h1 @ t["fc_2/kernel"] + t["fc_2/bias"])
    logits = h2 @ t["fc_out/kernel"] + t["fc_out/bias"]
    g1 = torch.tanh(x @ t["fc_value_1/kernel"] + t["fc_value_1/bias"])
    g2 = torch.tanh(g1 @ t["fc_value_2/kernel"] + t["fc_value_2/bias"])
    v = (g2 @ t["value_out/kernel"] + t["value_out/bias"])[:, 0]
    return t, _torch_ppo_loss(logits, v, batch, beta, cfg)


def _torch_ppo_loss(logits, v, batch, beta, cfg):
    T = lambda k: torch.tensor(batch[k], dtype=torch.float64)
    A = logits.shape[1] // 2
    mean, ls = logits[:, :A], logits[:, A:]
    a, ol = T("actions"), T("logits")
    logp = (-0.5 * (((a - mean) / ls.exp()) ** 2).sum(1) - 0.5 * np.log(2 * np.pi) * A
            - ls.sum(1))
    ratio = torch.exp(logp - T("logp"))
    adv = T("adv")
    surr = torch.minimum(adv * ratio, adv * torch.clamp(ratio, 0.8, 1.2))
    om, os_ = ol[:, :A], ol[:, A:]
    kl = (ls - os_ + (os_.exp() ** 2 + (om - mean) ** 2) / (2 * ls.exp() ** 2) - 0.5).sum(1)
    vf1 = (v - T("vt")) ** 2
    vf2 = (T("vf_preds") + torch.clamp(v - T("vf_preds"), -10, 10) - T("vt")) ** 2
    vf = torch.maximum(vf1, vf2)
    ent = (ls + 0.5 * np.log(2 * np.pi * np.e)).sum(1)
    return (-surr + beta * kl + 0.5 * vf - cfg.get("entropy_coeff", 0.0) * ent).mean()


def _rand_batch(rng, n, d, A=2, X=None):
    b = dict(actions=rng.normal(size=(n, A)).astype(np.float32),
             logits=np.concatenate([rng.normal(size=(n, A)) * 0.1,
                                    rng.normal(size=(n, A)) * 0.1 - 0.5], 1).astype(np.float32),
             vf_preds=rng.normal(size=n).astype(np.float32),
             adv=rng.normal(size=n).astype(np.float32),
             vt=rng.normal(size=n).astype(np.float32))
    b["logp"] = O.dg_logp(b["logits"], b["actions"]) + rng.normal(size=n).astype(np.float32) * 0.1
    if X is None:
        b["obs"] = rng.normal(size=(n, d)).astype(np.float32)
    return b


@pytest.mark.parametrize("d", [19, 35, 43])
def test_ffn_ppo_gradients_match_autograd(d):
    rng = np.random.default_rng(d)
    A = 8 if d == 43 else 2
    p = O.ffn_init(rng, d, 2 * A)
    # make the output heads non-trivial so every branch carries gradient
    p["fc_out/kernel"] *= 30
    p["value_out/kernel"] *= 30
    b = _rand_batch(rng, 128, d, A)
    beta, cfg = 0.3, {}
    logits, value, cache = O.ffn_forward(p, b["obs"])
    dl, dv, st = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"],
                                 b["vf_preds"], b["adv"], b["vt"], np.float32(beta))
    g = O.ffn_backward(p, cache, dl, dv)
    t, loss = _torch_ffn_loss(p, b, beta, cfg)
    loss.backward()
    assert abs(loss.item() - st["total_loss"]) < 1e-5 * max(1, abs(loss.item()))
    for k in p:
        ref = t[k].grad.numpy()
        np.testing.assert_allclose(g[k], ref, rtol=1e-4, atol=2e-5 * np.abs(ref).max(), err_msg=k)


def test_cup_gradients_match_autograd():
    """"cup" (models/coupling_net_glorot_uniform_init.py:22-30): coupled means, including
    the gradient of the trainable leg-coupling table, against torch autograd."""
    rng = np.random.default_rng(7)
    d, A, n = 19, 2, 128
    p = O.cup_init(rng, d, A)
    np.testing.assert_array_equal(p["leg_coupling"], [[1, 1], [-1, -1], [-1, -1], [1, 1]])
    p["leg_coupling"] = p["leg_coupling"] * rng.uniform(0.5, 1.5, size=(4, A)).astype(np.float32)
    p["fc_out/kernel"] *= 30
    p["value_out/kernel"] *= 30
    b = _rand_batch(rng, n, d, A)
    leg = rng.integers(0, 4, size=n)
    beta = 0.3
    logits, value, cache = O.cup_forward(p, b["obs"], leg)
    dl, dv, st = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"],
                                 b["vf_preds"], b["adv"], b["vt"], np.float32(beta))
    g = O.cup_backward(p, cache, dl, dv)
    t = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in p.items()}
    x = torch.tensor(b["obs"], dtype=torch.float64)
    h2 = torch.tanh(torch.tanh(x @ t["fc_1/kernel"] + t["fc_1/bias"]) @ t["fc_2/kernel"] + t["fc_2/bias"])
    raw = h2 @ t["fc_out/kernel"] + t["fc_out/bias"]
    coef = torch.cat([t["leg_coupling"], torch.ones(4, A, dtype=torch.float64)], 1)[torch.tensor(leg)]
    g2 = torch.tanh(torch.tanh(x @ t["fc_value_1/kernel"] + t["fc_value_1/bias"]) @ t["fc_value_2/kernel"]
                    + t["fc_value_2/bias"])
    v = (g2 @ t["value_out/kernel"] + t["value_out/bias"])[:, 0]
    loss = _torch_ppo_loss(raw * coef, v, b, beta, {})
    loss.backward()
    assert abs(loss.item() - st["total_loss"]) < 1e-5 * max(1, abs(loss.item()))
    assert np.abs(g["leg_coupling"]).max() > 0
    for k in p:
        ref = t[k].grad.numpy()
        np.testing.assert_allclose(g[k], ref, rtol=1e-4, atol=2e-5 * np.abs(ref).max(), err_msg=k)


def test_gnn_gradients_match_autograd():
    rng = np.random.default_rng(5)
    p = O.gnn_init(rng, 4)
    p["actor/linear_out/kernel"] *= 30
    p["critic/linear_out/kernel"] *= 30
    n = 32
    X = rng.normal(size=(n, 4, 23)).astype(np.float32)
    node = rng.integers(0, 4, size=n)
    b = _rand_batch(rng, n, 0, 2, X=True)
    logits, value, cache = O.gnn_forward(p, X, node)
    dl, dv, st = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"],
                                 b["vf_preds"], b["adv"], b["vt"], np.float32(0.2))
    g = O.gnn_backward(p, cache, dl, dv)

    t = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in p.items()}
    adj = torch.tensor(O.ring_adjacency())
    Xt = torch.tensor(X, dtype=torch.float64)

    def net(pre):
        f, q = Xt[..., :19], Xt[..., 19:]
        wn = torch.tanh(q @ t[pre + "state_enc/kernel"] + t[pre + "state_enc/bias"])
        wn = wn.reshape(n, 4, 19, 64)
        h = torch.tanh(torch.einsum("bni,bnij->bnj", f, wn))
        msg = h @ t[pre + "mpnn/msg_transform/kernel"]
        m = torch.einsum("sr,bsj->brj", adj, msg) / adj.sum(0)[None, :, None]
        y = torch.tanh(h @ t[pre + "mpnn/node_update/kernel"] + m)
        ys = y[torch.arange(n), torch.tensor(node)]
        return ys @ t[pre + "linear_out/kernel"] + t[pre + "linear_out/bias"]

    loss = _torch_ppo_loss(net("actor/"), net("critic/")[:, 0], b, 0.2, {})
    loss.backward()
    assert abs(loss.item() - st["total_loss"]) < 1e-5 * max(1, abs(loss.item()))
    for k in p:
        ref = t[k].grad.numpy()
        np.testing.assert_allclose(g[k], ref, rtol=1e-4, atol=2e-5 * np.abs(ref).max(), err_msg=k)


def _torch_gnn_layer(layer, t, pre, x, adj):
    """The reference's layer call (models/gcn.py), literally: tf.where edge lists, gather_nd,
    unsorted_segment_mean / segment_softmax, scatter_nd -- written in torch, independent of the
    oracle's einsum formulation."""
    B, n, H = x.shape
    if layer == "gcn":                       # gcn.py:29-37, graph_ops.adj_norm
        an = torch.diag_embed(adj.sum(-1) ** -1.0) @ adj
        return torch.tanh((an @ x) @ t[pre + "gcn/linear/kernel"])
    if layer == "gat1":
        adj = torch.clamp(adj + torch.eye(n, dtype=adj.dtype)[None], max=1.0)
    ei = torch.nonzero(adj != 0)             # tf.where order: (batch, sender, receiver)
    b, snd, rcv = ei[:, 0], ei[:, 1], ei[:, 2]
    seg = rcv + b * n

    def seg_sum(v):
        out = torch.zeros((B * n,) + v.shape[1:], dtype=v.dtype)
        return out.index_add(0, seg, v)

    cnt = seg_sum(torch.ones(len(seg), dtype=x.dtype))
    if layer == "mpnn":                      # gcn.py:57-94
        msgs = seg_sum(x[b, snd] @ t[pre + "mpnn/msg_transform/kernel"]) / torch.clamp(cnt, min=1)[:, None]
        return torch.tanh(x @ t[pre + "mpnn/node_update/kernel"] + msgs.reshape(B, n, H))
    if layer == "mpnn2":                     # gcn.py:113-150
        e = torch.cat([x[b, snd], x[b, rcv]], -1) @ t[pre + "mpnn2/msg_transform/kernel"]
        m = (seg_sum(e) / torch.clamp(cnt, min=1)[:, None]).reshape(B, n, H)
        return torch.tanh(torch.cat([x, m], -1) @ t[pre + "mpnn2/node_update/kernel"])
    # gat1: gcn.py:171-206, graph_ops.segment_softmax
    z = x @ t[pre + "gat1/pre_att_linear/kernel"]
    att = torch.cat([z[b, snd], z[b, rcv]], -1) @ t[pre + "gat1/att_linear/kernel"]
    att = torch.nn.functional.leaky_relu(att, 0.2)
    ex = torch.exp(att)
    att = ex / seg_sum(ex)[seg]
    A = torch.zeros((B, n, n), dtype=x.dtype).index_put((b, snd, rcv), att[:, 0])
    return torch.tanh(A @ z)


@pytest.mark.parametrize("layer", O.GNN_LAYERS)
@pytest.mark.parametrize("graph", ["ring", "random"])
def test_gnn_layer_gradients_match_autograd(layer, graph):
    """f4: GraphNet with each message-passing layer of models/gcn.py (MPNN, GCN, MPNN2, GAT1):
    the oracle's forward and manual backward against torch autograd of the reference's call(),
    on the ring graph and on random directed graphs (every node with an in-edge)."""
    rng = np.random.default_rng(11)
    p = O.gnn_init(rng, 4, layer=layer)
    p["actor/linear_out/kernel"] *= 30
    p["critic/linear_out/kernel"] *= 30
    n = 24
    X = rng.normal(size=(n, 4, 23)).astype(np.float32)
    node = rng.integers(0, 4, size=n)
    if graph == "ring":
        adj = np.broadcast_to(O.ring_adjacency(), (n, 4, 4)).astype(np.float32)
    else:
        adj = (rng.random((n, 4, 4)) < 0.5).astype(np.float32)
        adj[:, np.arange(4), (np.arange(4) + 1) % 4] = 1.0    # every row and column non-empty
    b = _rand_batch(rng, n, 0, 2, X=True)
    logits, value, cache = O.gnn_forward(p, X, node, adj, layer=layer)
    dl, dv, st = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"],
                                 b["vf_preds"], b["adv"], b["vt"], np.float32(0.2))
    g = O.gnn_backward(p, cache, dl, dv)
    assert sorted(g) == sorted(p)

    t = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in p.items()}
    adj_t = torch.tensor(adj, dtype=torch.float64)
    Xt = torch.tensor(X, dtype=torch.float64)

    def net(pre):
        f, q = Xt[..., :19], Xt[..., 19:]
        wn = torch.tanh(q @ t[pre + "state_enc/kernel"] + t[pre + "state_enc/bias"]).reshape(n, 4, 19, 64)
        h = torch.tanh(torch.einsum("bni,bnij->bnj", f, wn))
        y = _torch_gnn_layer(layer, t, pre, h, adj_t)
        return y[torch.arange(n), torch.tensor(node)] @ t[pre + "linear_out/kernel"] + t[pre + "linear_out/bias"]

    la, lv = net("actor/"), net("critic/")
    np.testing.assert_allclose(logits, la.detach().numpy(), rtol=1e-4, atol=1e-5)
    loss = _torch_ppo_loss(la, lv[:, 0], b, 0.2, {})
    loss.backward()
    assert abs(loss.item() - st["total_loss"]) < 1e-5 * max(1, abs(loss.item()))
    for k in p:
        ref = t[k].grad.numpy()
        assert np.abs(ref).max() > 0, k
        np.testing.assert_allclose(g[k], ref, rtol=1e-4, atol=2e-5 * np.abs(ref).max(), err_msg=k)


def test_gae_matches_direct_recursion():
    rng = np.random.default_rng(1)
    T, C = 50, 7
    r = rng.normal(size=(T, C)).astype(np.float32)
    v = rng.normal(size=(T, C)).astype(np.float32)
    d = np.zeros((T, C), bool)
    d[17, 2] = d[49, 3] = d[0, 5] = True
    lv = rng.normal(size=C).astype(np.float32)
    adv, vt = O.gae_fragment(r, v, d, lv)
    g, lam = 0.99, 0.95
    for c in range(C):
        acc, nxt = 0.0, float(lv[c])
        for t in range(T - 1, -1, -1):
            if d[t, c]:
                acc, nxt = 0.0, 0.0
            delta = float(r[t, c]) + g * nxt - float(v[t, c])
            acc = delta + g * lam * acc
            nxt = float(v[t, c])
            assert abs(adv[t, c] - np.float32(acc)) <= 1e-6 * max(1, abs(acc))


def test_adam_first_step_is_signlike():
    a = O.Adam(4)
    th = a.apply(np.zeros(4, np.float32), np.array([1, -2, 1e-3, 0], np.float32))
    np.testing.assert_allclose(th[:3], [-3e-4, 3e-4, -3e-4], rtol=1e-3)
    assert th[3] == 0
    assert a.b1p == np.float32(np.float32(0.9) * np.float32(0.9))


def test_clip_by_global_norm():
    g = [np.array([3.0, 4.0], np.float32)]
    c, n = O.clip_by_global_norm(g, 0.5)
    assert abs(n - 5) < 1e-6 and abs(np.linalg.norm(c[0]) - 0.5) < 1e-6
    c, _ = O.clip_by_global_norm([np.array([0.1], np.float32)], 0.5)
    assert c[0][0] == np.float32(0.1)


def test_kl_schedule():
    assert O.update_kl(0.2, 0.03) == pytest.approx(0.3)
    assert O.update_kl(0.2, 0.001) == pytest.approx(0.1)
    assert O.update_kl(0.2, 0.01) == 0.2


def test_graph_observation_and_quaternion():
    rng = np.random.default_rng(2)
    raw = rng.normal(size=43)
    normed = rng.normal(size=43)
    idx = [L.get_obs_indices(['body', leg]) for leg in ('fl', 'hl', 'hr', 'fr')]
    X = O.graph_observation(raw, normed, idx)
    assert X.shape == (4, 23)
    # identity rotation in component slot w of q1 -> result equals q2 (up to ordering)
    q = O.quaternion_multiply([0, 0, 0, 1], [0, 0, np.sin(0.3), np.cos(0.3)])
    np.testing.assert_allclose(q, [0, 0, np.sin(0.3), np.cos(0.3)], atol=1e-12)
    adj = O.ring_adjacency()
    assert adj.sum() == 8 and (adj.sum(0) == 2).all()


def test_oracle_reproduces_golden_vectors():
    """The committed oracle vectors (tests/golden/oracle_golden.npz, made by
    tests/golden/make_oracle_golden.py) are reproduced from their stored inputs: forward,
    sampling, GAE + standardization, and one PPO minibatch (gradient, clip + Adam) for the
    fcnet, "cup" and GraphNet models."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz"))
    close = lambda a, b: np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-7)
    shapes = O.ffn_param_shapes(35, 4)
    p = O.unpack(z["ffn_params"], shapes)
    logits, value, _ = O.ffn_forward(p, z["ffn_obs"])
    close(logits, z["ffn_logits"])
    close(value, z["ffn_value"])
    act = O.dg_sample(logits, z["ffn_eps"])
    close(act, z["ffn_actions"])
    close(O.dg_logp(logits, act), z["ffn_logp"])
    adv, vt = O.gae_fragment(z["gae_rew"], z["gae_vf"], z["gae_dones"], z["gae_last_v"])
    close(adv, z["gae_adv"])
    close(vt, z["gae_vt"])
    _, mean, std = O.standardize(adv.reshape(-1))
    close(np.array([mean, max(np.float32(1e-4), std)], np.float32), z["gae_norm"])
    for model, pre, shp in (("ffn", "ffn_step_", shapes), ("cup", "cup_", O.cup_param_shapes(19, 2)),
                            ("gnn", "gnn_", O.gnn_param_shapes(4))):
        params = O.unpack(z[pre + "params"] if model == "ffn" else z[pre + "params"], shp)
        b = {k[len(pre):]: z[k] for k in z.files if k.startswith(pre)}
        if model == "ffn":
            logits, value, cache = O.ffn_forward(params, b["obs"])
        elif model == "cup":
            logits, value, cache = O.cup_forward(params, b["obs"], b["leg"])
            close(logits, z["cup_fwd_logits"])
        else:
            logits, value, cache = O.gnn_forward(params, b["X"], b["node_idx"])
            close(logits, z["gnn_fwd_logits"])
            close(value, z["gnn_fwd_value"])
        dl, dv, st = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"], b["vf_preds"],
                                     b["adv"], b["vt"], np.float32(0.3 if model == "ffn" else 0.2))
        g = {"ffn": O.ffn_backward, "cup": O.cup_backward, "gnn": O.gnn_backward}[model](params, cache, dl, dv)
        flat = np.concatenate([g[n].reshape(-1) for n, _ in shp])
        close(flat, z[pre + "grad"])
        clipped, gn = O.clip_by_global_norm([flat], 0.5)
        new = O.Adam(flat.size).apply(O.pack(params, shp), clipped[0])
        close(new, z[pre + "new_params"])
        close(np.array([st["total_loss"], st["policy_loss"], st["vf_loss"], st["kl"], st["entropy"],
                        st["vf_explained_var"], gn], np.float32), z[pre + "stats"])


def test_ppo_branches_and_forced_decisions():
    """The tie-following trajectory's oracle hooks (tests/gpu_harness.tie_following_trajectory):
    ppo_branches reports each row's two clip decisions consistently with ppo_loss_rows' gradient
    (a row whose surrogate / value term is 'off' has zero d_ratio / d_vf), forcing every row to its
    own decision changes nothing bit for bit, and flipping one row's decision changes only that
    row's output gradient."""
    rng = np.random.default_rng(3)
    n, A = 64, 2
    logits = np.concatenate([rng.normal(size=(n, A)) * 0.3, rng.normal(size=(n, A)) * 0.2 - 0.5], 1).astype(np.float32)
    old = logits + rng.normal(size=logits.shape).astype(np.float32) * 0.3
    act = rng.normal(size=(n, A)).astype(np.float32)
    old_logp = O.dg_logp(old, act)
    vf_old = rng.normal(size=n).astype(np.float32) * 5
    value = (vf_old + rng.normal(size=n) * 12).astype(np.float32)
    vt = (vf_old + rng.normal(size=n) * 8).astype(np.float32)
    vt[::2] = value[::2] + rng.normal(size=n // 2).astype(np.float32)   # near V: clipped rows lose
    adv = rng.normal(size=n).astype(np.float32)
    args = (logits, value, act, old, old_logp, vf_old, adv, vt, np.float32(0.2))
    dl, dv, _ = O.ppo_loss_rows(*args)
    pol_on, pol_m, vf_on, m_sq, m_in = O.ppo_branches(logits, value, act, old_logp, vf_old, adv, vt)
    assert 0 < pol_on.sum() < n and 0 < vf_on.sum() < n       # both kinds of decision occur
    assert np.all(dv[~vf_on] == 0) and np.all(dv[vf_on] != 0)
    # the policy term's share of dlogits vanishes exactly when the surrogate is clipped (beta-only rows)
    dl_nokl, _, _ = O.ppo_loss_rows(*args[:-1], np.float32(0.0))
    assert np.all(dl_nokl[~pol_on] == 0) and np.all(np.abs(dl_nokl[pol_on]).sum(1) > 0)
    assert np.all((pol_m >= 0) == pol_on) and np.all(((m_sq >= 0) | (m_in >= 0)) == vf_on)
    same = {"pol": {i: bool(pol_on[i]) for i in range(n)}, "vf": {i: bool(vf_on[i]) for i in range(n)}}
    dl2, dv2, _ = O.ppo_loss_rows(*args, force=same)
    np.testing.assert_array_equal(dl2, dl)
    np.testing.assert_array_equal(dv2, dv)
    i = int(np.flatnonzero(~vf_on)[0])
    j = int(np.flatnonzero(pol_on)[0])
    dl3, dv3, _ = O.ppo_loss_rows(*args, force={"vf": {i: True}, "pol": {j: False}})
    assert dv3[i] != 0 and np.array_equal(np.delete(dv3, i), np.delete(dv, i))
    assert not np.array_equal(dl3[j], dl[j]) and np.array_equal(np.delete(dl3, j, 0), np.delete(dl, j, 0))
