"""Golden input/output vectors of the CPU oracle (SURVEY 8(c) fixture plan, item iii).

Seeded inputs and the oracle's outputs for every piece of the hot path, committed as
tests/golden/oracle_golden.npz:

  * fcnet (Local, d = 35, A = 2): rollout forward, DiagGaussian sample and logp of 64 rows;
    one PPO minibatch (128 rows): loss statistics, the flat gradient, the parameters after
    clip_by_global_norm + tf1 Adam;
  * GAE over a [T = 16, C = 8] fragment with episode ends, and StandardizeFields;
  * "cup" (d = 19, A = 2): coupled forward and the gradient of one minibatch;
  * GraphNet (gnn): forward and the gradient of one 128-row minibatch.

The fixtures pin the oracle itself (tests/test_oracle.py recomputes them) and give the HIP
path fixed targets (tests/test_gpu_golden.py).  Regenerate with

    python tests/golden/make_oracle_golden.py

The oracle follows the reference's algorithms (oracle/ddrl_oracle.py header: RLlib 1.0.1 /
TF 2.3.1 pieces restated, parity with those libraries unpinned); this script imports no
reference code.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ddrl_oracle as O  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle_golden.npz")
F = np.float32


def _batch(rng, n, d, A, logits_fn):
    obs = rng.normal(size=(n, d)).astype(F)
    old = logits_fn(obs)
    act = O.dg_sample(old, rng.normal(size=(n, A)).astype(F))
    return dict(obs=obs, actions=act, logits=old, logp=O.dg_logp(old, act),
                vf_preds=rng.normal(size=n).astype(F), adv=rng.normal(size=n).astype(F),
                vt=rng.normal(size=n).astype(F))


def _step(model, params, shapes, batch, kl, extra=None):
    """One minibatch of PPO: stats, flat gradient, parameters after clip + Adam."""
    fwd = {"ffn": lambda p, b: O.ffn_forward(p, b["obs"]),
           "cup": lambda p, b: O.cup_forward(p, b["obs"], b["leg"]),
           "gnn": lambda p, b: O.gnn_forward(p, b["X"], b["node_idx"])}[model]
    bwd = {"ffn": O.ffn_backward, "cup": O.cup_backward, "gnn": O.gnn_backward}[model]
    logits, value, cache = fwd(params, batch)
    dl, dv, st = O.ppo_loss_rows(logits, value, batch["actions"], batch["logits"], batch["logp"],
                                 batch["vf_preds"], batch["adv"], batch["vt"], F(kl))
    g = bwd(params, cache, dl, dv)
    flat_g = np.concatenate([g[n].reshape(-1) for n, _ in shapes]).astype(F)
    clipped, gn = O.clip_by_global_norm([flat_g], 0.5)
    adam = O.Adam(flat_g.size)
    new = adam.apply(O.pack(params, shapes), clipped[0])
    stats = np.array([st["total_loss"], st["policy_loss"], st["vf_loss"], st["kl"], st["entropy"],
                      st["vf_explained_var"], gn], F)
    return flat_g, new.astype(F), stats


def main():
    rng = np.random.default_rng(2024)
    out = {}
    # ---- fcnet, Local policy (d = 35, A = 2) ----
    d, A = 35, 2
    p = O.ffn_init(rng, d, 2 * A)
    p["fc_out/kernel"] *= 30          # non-trivial heads (as the GPU rollout tests)
    p["value_out/kernel"] *= 30
    p["fc_out/bias"] += np.array([0, 0, -0.5, -0.5], F)
    shapes = O.ffn_param_shapes(d, 2 * A)
    out["ffn_params"] = O.pack(p, shapes)
    x = rng.normal(size=(64, d)).astype(F)
    eps = rng.normal(size=(64, A)).astype(F)
    logits, value, _ = O.ffn_forward(p, x)
    act = O.dg_sample(logits, eps)
    out.update(ffn_obs=x, ffn_eps=eps, ffn_logits=logits, ffn_value=value, ffn_actions=act,
               ffn_logp=O.dg_logp(logits, act))
    # one minibatch step at the reference's output-head scale (well conditioned in fp32)
    p1 = O.ffn_init(rng, d, 2 * A)
    p1["fc_out/bias"] += np.array([0, 0, -0.5, -0.5], F)
    b = _batch(rng, 128, d, A, lambda o: O.ffn_forward(p1, o)[0] + F(0.05) * rng.normal(size=(128, 2 * A)).astype(F))
    g, new, stats = _step("ffn", p1, shapes, b, 0.3)
    out["ffn_step_params"] = O.pack(p1, shapes)
    for k, v in b.items():
        out["ffn_step_" + k] = v
    out.update(ffn_step_grad=g, ffn_step_new_params=new, ffn_step_stats=stats)

    # ---- GAE + StandardizeFields over a fragment with episode ends ----
    T, C = 16, 8
    rew = rng.normal(size=(T, C)).astype(F)
    vf = rng.normal(size=(T, C)).astype(F)
    dones = rng.random(size=(T, C)) < 0.1
    last_v = rng.normal(size=C).astype(F)
    adv, vt = O.gae_fragment(rew, vf, dones, last_v)
    _, mean, std = O.standardize(adv.reshape(-1))
    out.update(gae_rew=rew, gae_vf=vf, gae_dones=dones, gae_last_v=last_v, gae_adv=adv, gae_vt=vt,
               gae_norm=np.array([mean, max(F(1e-4), std)], F))

    # ---- cup (d = 19, A = 2) ----
    pc = O.cup_init(rng, 19, 2)
    pc["leg_coupling"] = (pc["leg_coupling"] * rng.uniform(0.5, 1.5, size=(4, 2))).astype(F)
    pc["fc_out/bias"] += np.array([0, 0, -0.5, -0.5], F)
    cshapes = O.cup_param_shapes(19, 2)
    leg = rng.integers(0, 4, size=128)
    bc = _batch(rng, 128, 19, 2, lambda o: O.cup_forward(pc, o, leg)[0])
    bc["leg"] = leg
    g, new, stats = _step("cup", pc, cshapes, bc, 0.2)
    out["cup_params"] = O.pack(pc, cshapes)
    for k, v in bc.items():
        out["cup_" + k] = v
    out.update(cup_fwd_logits=O.cup_forward(pc, bc["obs"], leg)[0], cup_grad=g, cup_new_params=new,
               cup_stats=stats)

    # ---- GraphNet ----
    pg = O.gnn_init(rng, 4)
    for net in ("actor/", "critic/"):
        pg[net + "state_enc/bias"] += (rng.normal(size=pg[net + "state_enc/bias"].shape) * 0.2).astype(F)
    pg["actor/linear_out/bias"] += np.array([0, 0, -0.5, -0.5], F)
    gshapes = O.gnn_param_shapes(4)
    X = rng.normal(size=(128, 4, 23)).astype(F)
    node = rng.integers(0, 4, size=128)
    lg, vg, _ = O.gnn_forward(pg, X, node)
    bg = dict(X=X, node_idx=node)
    act = O.dg_sample(lg, rng.normal(size=(128, 2)).astype(F))
    bg.update(actions=act, logits=(lg + F(0.05) * rng.normal(size=lg.shape)).astype(F),
              vf_preds=rng.normal(size=128).astype(F), adv=rng.normal(size=128).astype(F),
              vt=rng.normal(size=128).astype(F))
    bg["logp"] = O.dg_logp(bg["logits"], act)
    g, new, stats = _step("gnn", pg, gshapes, bg, 0.2)
    out["gnn_params"] = O.pack(pg, gshapes)
    for k, v in bg.items():
        out["gnn_" + k] = v
    out.update(gnn_fwd_logits=lg, gnn_fwd_value=vg, gnn_grad=g, gnn_new_params=new, gnn_stats=stats)

    np.savez_compressed(OUT, **out)
    print(OUT, os.path.getsize(OUT), "bytes,", len(out), "arrays")


if __name__ == "__main__":
    main()
