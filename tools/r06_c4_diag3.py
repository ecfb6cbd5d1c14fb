"""VERDICT r05 item 1, third pass: which row of step K's minibatch does the HIP gradient treat
differently?  From the numpy fp32 state after K steps: the HIP gradient (ddrl_ppo_grad) against
the fp64 gradient with one row's value (or policy) term removed or switched, and that row's
per-row quantities in fp32 / fp64.  Test infrastructure: imports the oracle.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from oracle import ddrl_oracle as O  # noqa: E402
import r06_c4_diag as D  # noqa: E402

K = int(os.environ.get("K", "679"))


def main():
    import torch
    from ddrl_amd.synthetic import SyntheticRollout
    from tests.gpu_harness import init_params, make_ctx

    ctx, cfg, inst = make_ctx(D.ENV, D.NENV, D.T)
    params = init_params(ctx, cfg, 13, head_scale=1.0)[0]
    syn = SyntheticRollout(D.NENV, D.T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=13)
    done = syn.dones_for_fragment()
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, done, syn.actions)
    ctx.gae()
    ctx.synchronize()
    del syn
    rec = ctx.records_get(0)
    lay = ctx.layout[0]
    d, A = cfg.obs_dim[0], cfg.act_dim
    mean, den = ctx.adv_norm_get(0)
    batch = dict(obs=rec[:, :d], actions=rec[:, lay["act"]:lay["act"] + A],
                 logits=rec[:, lay["logit"]:lay["logit"] + 2 * A], logp=rec[:, lay["logp"]],
                 vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                 vt=rec[:, lay["vt"]])
    shapes = O.ffn_param_shapes(d, 2 * A)
    theta0 = O.pack(params, shapes)
    n = theta0.size
    R = rec.shape[0]
    sh, pe = O.sgd_schedule(np.random.default_rng(44), R, 128, 10)
    rows_of = lambda k: sh[pe[0, k] * 128:(pe[0, k] + 1) * 128]
    O64 = O.with_dtype(np.float64)
    st = D.State(O, theta0, n)
    for k in range(K):
        D.one_step(st, shapes, batch, rows_of(k), 0.2)
    rows = rows_of(K)
    print(f"step {K}: rows {rows.min()}..{rows.max()}, layout {lay}", flush=True)

    r = torch.from_numpy(np.ascontiguousarray(rows)).cuda()
    gbuf = torch.zeros(n, device="cuda")
    ctx.params_set(0, st.theta)
    ctx.ppo_grad(0, r, 128, 0.2, gbuf, 0)
    ctx.synchronize()
    gh = gbuf.cpu().numpy().astype(np.float64)
    sth = ctx.ppo_stats(0, 1)[0]

    p64 = {k: v.astype(np.float64) for k, v in O.unpack(st.theta, shapes).items()}
    logits, value, cache = O64.ffn_forward(p64, batch["obs"][rows])
    args = (batch["actions"][rows], batch["logits"][rows], batch["logp"][rows], batch["vf_preds"][rows],
            batch["adv"][rows], batch["vt"][rows])
    dl, dv, s64 = O64.ppo_loss_rows(logits, value, *args, np.float64(0.2))
    g = O64.ffn_backward(p64, cache, dl, dv)
    g64 = np.concatenate([g[nm_].reshape(-1) for nm_, _ in shapes])
    print(f"HIP stats {sth}", flush=True)
    print(f"fp64 stats {s64}", flush=True)
    base = np.abs(gh - g64).max()
    o = 0
    for nm_, shp in shapes:
        k_ = int(np.prod(shp))
        e_ = gh[o:o + k_] - g64[o:o + k_]
        print(f"  {nm_:20s} max|err| {np.abs(e_).max():.4g}  max|g64| {np.abs(g64[o:o + k_]).max():.4g}", flush=True)
        o += k_
    # value-branch error explained by per-row dvalue changes?  J_i = the value-parameter gradient
    # of a unit dvalue on row i
    vsel = np.concatenate([np.full(int(np.prod(s_)), nm_.startswith(("fc_value", "value_out"))) for nm_, s_ in shapes])
    psel = ~vsel
    J = []
    for i in range(128):
        u = np.zeros(128)
        u[i] = 1.0
        gg = O64.ffn_backward(p64, cache, np.zeros_like(dl), u)
        J.append(np.concatenate([gg[nm_].reshape(-1) for nm_, _ in shapes])[vsel])
    J = np.array(J).T
    ev = (gh - g64)[vsel]
    delta, *_ = np.linalg.lstsq(J, ev, rcond=None)
    res = np.abs(J @ delta - ev).max()
    big = np.argsort(-np.abs(delta))[:8]
    print(f"value error as per-row dvalue changes: residual {res:.3g} of {np.abs(ev).max():.3g}; largest "
          + ", ".join(f"row {i}: d_dvalue {delta[i]:.4g} (dvalue {dv[i]:.4g})" for i in big), flush=True)
    Jp = []
    for i in range(128):
        for j in range(dl.shape[1]):
            u = np.zeros_like(dl)
            u[i, j] = 1.0
            gg = O64.ffn_backward(p64, cache, u, np.zeros(128))
            Jp.append(np.concatenate([gg[nm_].reshape(-1) for nm_, _ in shapes])[psel])
    Jp = np.array(Jp).T
    ep = (gh - g64)[psel]
    dp_, *_ = np.linalg.lstsq(Jp, ep, rcond=None)
    resp = np.abs(Jp @ dp_ - ep).max()
    bigp = np.argsort(-np.abs(dp_))[:8]
    print(f"policy error as per-row dlogits changes: residual {resp:.3g} of {np.abs(ep).max():.3g}; largest "
          + ", ".join(f"row {i // dl.shape[1]} out {i % dl.shape[1]}: {dp_[i]:.4g} (dlogit {dl.reshape(-1)[i]:.4g})" for i in bigp), flush=True)
    print(f"max |g_hip - g64| = {base:.4g}", flush=True)

    def gwith(dl_, dv_):
        gg = O64.ffn_backward(p64, cache, dl_, dv_)
        return np.concatenate([gg[nm_].reshape(-1) for nm_, _ in shapes])

    best = []
    for i in range(128):
        dv2 = dv.copy()
        dv2[i] = 0.0
        e_v = np.abs(gh - gwith(dl, dv2)).max()
        dl2 = dl.copy()
        dl2[i] = 0.0
        e_p = np.abs(gh - gwith(dl2, dv)).max()
        best.append((min(e_v, e_p), i, e_v, e_p))
    best.sort()
    print("rows whose removal brings fp64 closest to HIP (err, row, value-term removed, policy-term removed):",
          best[:4], flush=True)
    i = best[0][1]
    ri = rows[i]
    f = np.float32
    V32 = f(O.ffn_forward(O.unpack(st.theta, shapes), batch["obs"][rows])[1][i])
    vfo, vt = f(batch["vf_preds"][ri]), f(batch["vt"][ri])
    dvv = f(V32 - vfo)
    vcl = f(vfo + np.clip(dvv, f(-10), f(10)))
    print(f"row {i} (record {ri}): V fp64 {value[i]:.9g} fp32 {V32:.9g}; vf_old {vfo:.9g}; vt {vt:.9g}; "
          f"dv {dvv:.9g}; vcl {vcl:.9g}; vf1 {f((V32 - vt) ** 2):.9g} vf2 {f((vcl - vt) ** 2):.9g}; "
          f"dvalue fp64 {dv[i]:.6g}; adv {batch['adv'][ri]:.6g}; logits {batch['logits'][ri]}; "
          f"logp_old {batch['logp'][ri]:.6g}; actions {batch['actions'][ri]}", flush=True)
    print(f"record row {ri} raw: {rec[ri]}", flush=True)
    print(f"the row's obs: {batch['obs'][ri]}", flush=True)
    # the same row alone through the HIP gradient and fp64
    for sub in ([i], [j for j in range(128) if j != i]):
        rr = torch.from_numpy(np.ascontiguousarray(rows[sub])).cuda()
        ctx.ppo_grad(0, rr, len(sub), 0.2, gbuf, 0)
        ctx.synchronize()
        gs = gbuf.cpu().numpy().astype(np.float64)
        lg, vv, cc = O64.ffn_forward(p64, batch["obs"][rows[sub]])
        a2 = tuple(x[sub] for x in args)
        dl_, dv_, _ = O64.ppo_loss_rows(lg, vv, *a2, np.float64(0.2))
        # the kernel scales by 1 / sgd_minibatch_size, ppo_loss_rows by 1 / rows
        gg = O64.ffn_backward(p64, cc, dl_ * len(sub) / 128, dv_ * len(sub) / 128)
        g2 = np.concatenate([gg[nm_].reshape(-1) for nm_, _ in shapes])
        print(f"  rows {'[i]' if len(sub) == 1 else 'all but i'}: max |g_hip - g64| {np.abs(gs - g2).max():.4g} "
              f"(max |g64| {np.abs(g2).max():.4g}); HIP stats {ctx.ppo_stats(0, 1)[0]}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
