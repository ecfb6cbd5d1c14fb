"""VERDICT r05 item 1, second pass: the step where the HIP C4 trajectory leaves fp64 (found at
H = 680 by tools/r06_c4_diag.py), taken apart parameter by parameter.

From the numpy fp32 state after k steps (k in a window around the departure):
  * the gradient of step k's minibatch from ddrl_ppo_grad (row split, the pair path), from a
    DDRL_UPDATE_SPLIT=1 context (no row split), numpy fp32 and numpy fp64;
  * one fused HIP step vs numpy fp32 / fp64 from the same state;
and, for the parameters whose HIP step deviates most, the gradient values, Adam's sqrt(v) and
the per-row contributions' magnitude (sum |row terms|, the scale of any summation error).
Test infrastructure: imports the oracle.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from oracle import ddrl_oracle as O  # noqa: E402
import r06_c4_diag as D  # noqa: E402

K0, K1 = int(os.environ.get("K0", "672")), int(os.environ.get("K1", "684"))


def grads(mod, theta, shapes, batch, rows, kl=0.2):
    F = mod.F32
    p = mod.unpack(np.asarray(theta, F), shapes)
    logits, value, cache = mod.ffn_forward(p, batch["obs"][rows])
    dl, dv, _ = mod.ppo_loss_rows(logits, value, batch["actions"][rows], batch["logits"][rows],
                                  batch["logp"][rows], batch["vf_preds"][rows], batch["adv"][rows],
                                  batch["vt"][rows], F(kl))
    g = mod.ffn_backward(p, cache, dl, dv)
    # magnitude of the per-row terms: the same backward with |.| everywhere (an upper scale of
    # any summation error: sum over rows of |row term|)
    return np.concatenate([g[n].reshape(-1) for n, _ in shapes]).astype(np.float64), (p, cache, dl, dv)


def abs_scale(p, cache, dl, dv, shapes):
    x, h1, h2, g1, g2 = [np.abs(np.asarray(c, np.float64)) for c in cache]
    P = {k: np.abs(np.asarray(v, np.float64)) for k, v in p.items()}
    dl, dv = np.abs(np.asarray(dl, np.float64)), np.abs(np.asarray(dv, np.float64))[:, None]
    g = {}
    g["fc_out/kernel"], g["fc_out/bias"] = h2.T @ dl, dl.sum(0)
    dz2 = (dl @ P["fc_out/kernel"].T) * np.abs(1 - h2 * h2)
    g["fc_2/kernel"], g["fc_2/bias"] = h1.T @ dz2, dz2.sum(0)
    dz1 = (dz2 @ P["fc_2/kernel"].T) * np.abs(1 - h1 * h1)
    g["fc_1/kernel"], g["fc_1/bias"] = x.T @ dz1, dz1.sum(0)
    g["value_out/kernel"], g["value_out/bias"] = g2.T @ dv, dv.sum(0)
    dy2 = (dv @ P["value_out/kernel"].T) * np.abs(1 - g2 * g2)
    g["fc_value_2/kernel"], g["fc_value_2/bias"] = g1.T @ dy2, dy2.sum(0)
    dy1 = (dy2 @ P["fc_value_2/kernel"].T) * np.abs(1 - g1 * g1)
    g["fc_value_1/kernel"], g["fc_value_1/bias"] = x.T @ dy1, dy1.sum(0)
    return np.concatenate([g[n].reshape(-1) for n, _ in shapes])


def names(shapes):
    out = []
    for n, s in shapes:
        for idx in np.ndindex(*s):
            out.append(f"{n}{list(idx)}")
    return out


def main():
    import torch
    from ddrl_amd import native as N
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
    nm = names(shapes)
    theta0 = O.pack(params, shapes)
    n = theta0.size
    R = rec.shape[0]
    sh, pe = O.sgd_schedule(np.random.default_rng(44), R, 128, 10)
    rows_of = lambda k: sh[pe[0, k] * 128:(pe[0, k] + 1) * 128]
    O64 = O.with_dtype(np.float64)

    os.environ["DDRL_UPDATE_SPLIT"] = "1"
    ctx1 = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
    del os.environ["DDRL_UPDATE_SPLIT"]
    ctx1.records_set(0, rec)
    ctx1.adv_norm_set(0, mean, den)

    st = D.State(O, theta0, n)
    dsh = torch.from_numpy(sh).cuda()
    gbuf = torch.zeros(n, device="cuda")
    inv = np.float64(1.0 / 128)
    print("per step k: max |g - g64| / sum|row terms| for the pair path (split 2), split 1, numpy fp32;"
          " and the one-step theta deviation", flush=True)
    for k in range(K1 + 1):
        if k >= K0:
            rows = rows_of(k)
            g64, (p, cache, dl, dv) = grads(O64, st.theta.astype(np.float64), shapes, batch, rows)
            g32, _ = grads(O, st.theta, shapes, batch, rows)
            scale = abs_scale(p, cache, dl, dv, shapes) + 1e-30
            r = torch.from_numpy(np.ascontiguousarray(rows)).cuda()
            gh = {}
            for key, c in (("split2", ctx), ("split1", ctx1)):
                c.params_set(0, st.theta)
                c.ppo_grad(0, r, 128, 0.2, gbuf)
                c.synchronize()
                gh[key] = gbuf.cpu().numpy().astype(np.float64)
            e = {key: np.abs(v - g64) / scale for key, v in list(gh.items()) + [("fp32", g32)]}
            # one fused step from the same state
            s64 = D.State(O64, st.theta.astype(np.float64), n)
            s64.adam.m, s64.adam.v = st.adam.m.astype(np.float64), st.adam.v.astype(np.float64)
            s64.adam.b1p, s64.adam.b2p = np.float64(st.adam.b1p), np.float64(st.adam.b2p)
            D.one_step(s64, shapes, batch, rows, 0.2)
            s32 = st.copy()
            D.one_step(s32, shapes, batch, rows, 0.2)
            pek = pe.copy()
            pek[0, 0] = pe[0, k]
            ctx.params_set(0, st.theta)
            ctx.adam_set(0, st.adam.m, st.adam.v, float(st.adam.b1p), float(st.adam.b2p))
            ctx.ppo_update(1, [dsh], [torch.from_numpy(pek).cuda()], [0.2], max_steps=1)
            ctx.synchronize()
            th_h = ctx.params_get(0).astype(np.float64)
            dh, d32 = np.abs(th_h - s64.theta), np.abs(s32.theta - s64.theta)
            print(f"k={k}: grad err/scale split2 {e['split2'].max():.3g} split1 {e['split1'].max():.3g} "
                  f"fp32 {e['fp32'].max():.3g} | step dev HIP {dh.max():.3g} fp32 {d32.max():.3g}", flush=True)
            if dh.max() > 1e-6 or d32.max() > 1e-6:
                top = np.argsort(-dh)[:6]
                sv = np.sqrt(st.adam.v.astype(np.float64))
                for i in top:
                    print(f"    {nm[i]:28s} dtheta HIP {dh[i]:.3g} fp32 {d32[i]:.3g} | g64 {g64[i]:.4g} "
                          f"split2 {gh['split2'][i]:.4g} split1 {gh['split1'][i]:.4g} fp32 {g32[i]:.4g} "
                          f"| sum|terms| {scale[i]:.3g} | m {st.adam.m[i]:.3g} sqrt(v) {sv[i]:.3g}", flush=True)
        D.one_step(st, shapes, batch, rows_of(k), 0.2)
    ctx1.close()
    ctx.close()


if __name__ == "__main__":
    main()
