"""Prototype of the tie-following parity check at C4: HIP against the fp64
trajectory that takes the kernel's outcome at near-tie clip decisions (tests/gpu_harness.py
tie_following_trajectory).  Test infrastructure: imports the oracle."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ddrl_oracle as O  # noqa: E402

HMAX = int(os.environ.get("HMAX", "6400"))
TOL = float(os.environ.get("TOL", "2e-5"))
HORIZONS = [h for h in (10, 100, 400, 680, 1000, 1600, 3200, 6400) if h <= HMAX]
t0 = time.time()


def log(*a):
    print(f"[{time.time() - t0:7.1f}s]", *a, flush=True)


def main():
    import torch
    from ddrl_amd.synthetic import SyntheticRollout
    from tests.gpu_harness import init_params, make_ctx, tie_following_trajectory

    ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_SharedDecentral", 4096, 200)
    params = init_params(ctx, cfg, 13, head_scale=1.0)[0]
    syn = SyntheticRollout(4096, 200, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=13)
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
    sh, pe = O.sgd_schedule(np.random.default_rng(44), rec.shape[0], 128, 10)
    O64 = O.with_dtype(np.float64)
    s64 = {h: None for h in HORIZONS}
    O64.ppo_update("ffn", {k: v.astype(np.float64) for k, v in params.items()}, shapes, O64.Adam(n), batch, sh, pe,
                   0.2, {}, steps=HMAX, snapshots=s64)
    s32 = {h: None for h in HORIZONS}
    O.ppo_update("ffn", params, shapes, O.Adam(n), batch, sh, pe, 0.2, {}, steps=HMAX, snapshots=s32)
    log("plain fp64 / fp32 done")
    tf, tst, ties = tie_following_trajectory(ctx, 0, params, shapes, batch, sh, pe, 0.2, HMAX, HORIZONS, tol=TOL,
                                             log=log)
    log(f"tie-following trajectory done: {len(ties)} ambiguous decisions, "
        f"{sum(t[4] != t[5] for t in ties)} taken the other way by HIP")
    dsh, dpe = torch.from_numpy(sh).cuda(), torch.from_numpy(pe).cuda()
    for H in HORIZONS:
        ctx.params_set(0, theta0)
        ctx.adam_set(0, np.zeros(n, np.float32), np.zeros(n, np.float32), 0.9, 0.999)
        ctx.ppo_update(1, [dsh], [dpe], [0.2], max_steps=H)
        ctx.synchronize()
        got = ctx.params_get(0).astype(np.float64)
        st = ctx.ppo_stats(0, H).astype(np.float64)
        e32 = np.abs(s32[H] - s64[H]).max()
        etf = np.abs(got - tf[H]).max()
        e64 = np.abs(got - s64[H]).max()
        e32tf = np.abs(s32[H] - tf[H]).max()
        sdev = {}
        for col, key in [(1, "policy_loss"), (2, "vf_loss"), (3, "kl"), (4, "entropy"), (6, "grad_gnorm")]:
            ref = np.array([s[key] for s in tst[:H]])
            sdev[key] = float(np.max(np.abs(st[:, col] - ref) / (np.abs(ref) + 1e-6)))
        log(f"H={H}: HIP - tie-following fp64 {etf:.3g} ({np.mean(np.abs(got - tf[H]) <= 1e-5):.4f} within 1e-5); "
            f"HIP - plain fp64 {e64:.3g}; numpy fp32 - plain fp64 {e32:.3g}, - tie-following {e32tf:.3g}; "
            f"stats max rel dev {', '.join(f'{k} {v:.2g}' for k, v in sdev.items())}")
    ctx.close()


if __name__ == "__main__":
    main()
