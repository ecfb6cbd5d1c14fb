"""ddrl_ppo_update_from (round 6): a fused update resumed at schedule step k from the state the
context holds is bit-identical to the same steps of one uninterrupted launch -- weights, Adam
moments, beta powers and learner statistics -- for every k mod 4 (the fused exchange's quad tag
bit follows the schedule step, and the resumed launch pre-fills each outbox with the complement
of its first bit), for the 4-policy fcnet launch (Local), the shared fcnet (C4) and the one-launch
GraphNet step (C5)."""
import numpy as np
import pytest

from tests.gpu_harness import GNN_ENV, init_gnn_params, init_params, make_ctx

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _setup(env, n, T, gnn):
    import torch
    from ddrl_amd.synthetic import SyntheticRollout
    ctx, cfg, _ = make_ctx(env, n, T)
    if gnn:
        init_gnn_params(ctx, 3, head_scale=1.0)
    else:
        init_params(ctx, cfg, 3, head_scale=1.0)
    syn = SyntheticRollout(n, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=5)
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, syn.dones_for_fragment(), syn.actions)
    ctx.gae()
    ctx.synchronize()
    P = cfg.n_policies
    rng = np.random.default_rng(9)
    sh, pe = [], []
    for p in range(P):
        R = T * ctx.layout[p]["C"]
        nb = R // 128
        sh.append(torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda())
        pe.append(torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(cfg.num_sgd_iter)])
                                   .astype(np.int32)).cuda())
    theta0 = [ctx.params_get(p) for p in range(P)]
    return ctx, cfg, sh, pe, theta0


def _reset(ctx, theta0):
    for p, th in enumerate(theta0):
        ctx.params_set(p, th)
        ctx.adam_set(p, np.zeros(th.size, np.float32), np.zeros(th.size, np.float32), 0.9, 0.999)


def _state(ctx, P, H):
    out = []
    for p in range(P):
        m, v, b1, b2 = ctx.adam_get(p)
        out += [ctx.params_get(p), m, v, np.array([b1, b2], np.float32), ctx.ppo_stats(p, H)]
    return out


@pytest.mark.parametrize("env,n,gnn", [("QuantrupedMultiEnv_Local", 32, False),
                                       ("QuantrupedMultiEnv_SharedDecentral", 16, False),
                                       (GNN_ENV, 16, True)])
def test_resumed_update_is_bit_identical(env, n, gnn):
    ctx, cfg, sh, pe, theta0 = _setup(env, n, 200, gnn)
    P = cfg.n_policies
    mask = (1 << P) - 1
    kl = [0.2] * P
    H = 41
    _reset(ctx, theta0)
    ctx.ppo_update(mask, sh, pe, kl, max_steps=H)
    ctx.synchronize()
    ref = _state(ctx, P, H)
    for k in (1, 2, 3, 4, 5, 6, 7, 13, 22):
        _reset(ctx, theta0)
        ctx.ppo_update(mask, sh, pe, kl, max_steps=k)
        ctx.ppo_update(mask, sh, pe, kl, max_steps=H - k, step0=k)
        ctx.synchronize()
        got = _state(ctx, P, H)
        for i, (a, b) in enumerate(zip(got, ref)):
            np.testing.assert_array_equal(a, b, err_msg=f"{env}: resumed at step {k}, item {i}")
    # three pieces, the last to the end of the schedule
    total = cfg.num_sgd_iter * (200 * ctx.layout[0]["C"] // 128)
    _reset(ctx, theta0)
    ctx.ppo_update(mask, sh, pe, kl)
    ctx.synchronize()
    ref = _state(ctx, P, total)
    _reset(ctx, theta0)
    ctx.ppo_update(mask, sh, pe, kl, max_steps=10)
    ctx.ppo_update(mask, sh, pe, kl, max_steps=27, step0=10)
    ctx.ppo_update(mask, sh, pe, kl, step0=37)
    ctx.synchronize()
    for i, (a, b) in enumerate(zip(_state(ctx, P, total), ref)):
        np.testing.assert_array_equal(a, b, err_msg=f"{env}: three pieces, item {i}")
    ctx.close()
