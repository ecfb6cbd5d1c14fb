"""The fused update's LSB-tagged exchange, bounded against the data-parallel gradient (VERDICT r4
item 7; DESIGN.md section 4, "Parity contract of the fused row split").

A fused launch (ddrl_ppo_update) splits each branch's 128-row minibatch over two workgroups
that swap their 64-row partial gradients every step.  Each exchanged partial carries a 1-bit
step tag in its own mantissa LSB (ppo_ffn_impl.h lx_t), and both workgroups add the two
LSB-replaced partials: g_fused = fl(lx(a) + lx(b)).  The data-parallel gradient launch
(ddrl_ppo_grad, the pair path) adds the same two partials untouched: g_pair = fl(a + b).  So
per parameter

    |g_fused - g_pair| <= ulp(a) + ulp(b) + ulp(g_pair)          (one ulp per partial + the sum)

The fused gradient is observed through Adam's first moment after one step from m = v = 0:
m1 = fl(fl(g * s) * (1 - beta1)), s = the step's clip scale (learner statistic 7).  The test
forms m1 of the pair gradient with the same s and requires, per parameter,

    |m1_fused - m1_pair| <= s (1 - beta1) (ulp(a) + ulp(b) + ulp(g_pair)) + 2 ulp(m1)

with |a|, |b| taken from the two 64-row halves' own gradient launches.  It also counts the
parameters whose fused and pair values differ (the perturbation is real, and bounded).
"""
import numpy as np
import pytest

from tests.gpu_harness import init_params, make_ctx, run_rollout

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ulp(x):
    x = np.abs(np.asarray(x, np.float32))
    return (np.nextafter(x, np.float32(np.inf)) - x).astype(np.float64)


@pytest.mark.parametrize("env", ["QuantrupedMultiEnv_Local", "QuantrupedMultiEnv_SharedDecentral"])
def test_fused_gradient_within_one_ulp_per_partial_of_pair_gradient(env):
    import torch
    ctx, cfg, inst = make_ctx(env, 32, 8)
    rng = np.random.default_rng(5)
    params = init_params(ctx, cfg, 9, head_scale=1.0)
    filt = (1000.0, rng.normal(size=cfg.obs_full_dim) * 0.3, np.abs(rng.normal(size=cfg.obs_full_dim)) * 999.0 + 10.0)
    run_rollout(ctx, cfg, inst, params, rng, filt, cfg.frag_len)
    P = cfg.n_policies
    sh, pe, rows = [], [], []
    for p in range(P):
        R = ctx.layout[p]["C"] * cfg.frag_len
        nb = R // 128
        s = rng.permutation(R).astype(np.int32)
        q = np.stack([rng.permutation(nb) for _ in range(cfg.num_sgd_iter)]).astype(np.int32)
        sh.append(torch.from_numpy(s).cuda())
        pe.append(torch.from_numpy(q).cuda())
        rows.append(s[q[0, 0] * 128:(q[0, 0] + 1) * 128].copy())
    # the pair path: the whole minibatch (row split, untouched partials) and its two halves
    g = {}
    for p in range(P):
        n = ctx.n_params[p]
        for key, r in (("full", rows[p]), ("a", rows[p][:64]), ("b", rows[p][64:])):
            buf = torch.zeros(n, device="cuda")
            ctx.ppo_grad(p, torch.from_numpy(np.ascontiguousarray(r)).cuda(), r.size, 0.2, buf)
            ctx.synchronize()
            g[p, key] = buf.cpu().numpy()
    # one fused step from m = v = 0 (clip + Adam of the LSB-replaced sums)
    for p in range(P):
        n = ctx.n_params[p]
        ctx.adam_set(p, np.zeros(n, np.float32), np.zeros(n, np.float32), 0.9, 0.999)
    ctx.ppo_update((1 << P) - 1, sh, pe, [0.2] * P, max_steps=1)
    ctx.synchronize()
    c1 = np.float32(1.0) - np.float32(cfg.adam_beta1)
    for p in range(P):
        s = np.float32(ctx.ppo_stats(p, 1)[0, 7])
        m1 = ctx.adam_get(p)[0].astype(np.float64)
        gp, ga, gb = g[p, "full"], g[p, "a"], g[p, "b"]
        m1p = ((gp * s).astype(np.float32) * c1).astype(np.float32).astype(np.float64)
        bound = float(s) * float(c1) * (_ulp(ga) + _ulp(gb) + _ulp(gp)) + 2 * _ulp(m1p)
        dev = np.abs(m1 - m1p)
        differ = int(np.sum(m1 != m1p))
        worst = float(np.max(dev / np.maximum(bound, 1e-45)))
        print(f"\n{env} policy {p}: {differ} of {m1.size} first moments differ from the pair path's; "
              f"worst deviation / bound {worst:.3f}")
        assert np.all(dev <= bound), (p, np.flatnonzero(dev > bound)[:10], worst)
        assert np.isfinite(m1).all()
    ctx.close()
