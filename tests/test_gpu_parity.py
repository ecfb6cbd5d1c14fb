"""HIP path vs CPU oracle through the C-ABI (needs an MI355X).

Tolerances (fp32 path, float64 filter/GAE as in the reference):
  * rollout outputs, rewards, GAE, gradients, losses: |gpu - ref| <= 1e-5 + 1e-5 |ref|
    (gradients: relative to the tensor's max magnitude, see _close_grad)
  * learner tests use the reference's own output-head scale (Glorot 0.01): with heads
    scaled up 30x (used for the rollout tests) log_std gets small enough that the loss is
    ill-conditioned and fp32 summation-order differences reach 2e-4 relative
  * parameters after Adam steps: 1e-5 absolute for >= 99.9 % of the entries; the rest
    (gradients within rounding of zero, where Adam's m / sqrt(v) flips sign) within
    2 * lr per step.
"""
import numpy as np
import pytest

from ddrl_amd import native as N
from oracle import ddrl_oracle as O
from tests.gpu_harness import init_params, make_ctx, run_rollout, strict_params_check

pytestmark = pytest.mark.gpu
RT, AT = 1e-5, 1e-5


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


def _close(a, b, rtol=RT, atol=AT, msg=""):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=msg)


def _filt(D, rng):
    return (1000.0, rng.normal(size=D) * 0.3, np.abs(rng.normal(size=D)) * 999.0 + 10.0)


ROLLOUT_ENVS = [
    ("QuantrupedMultiEnv_Local", 64, 6),
    ("QuantrupedMultiEnv_FullyDecentral", 40, 5),
    ("QuantrupedMultiEnv_SharedDecentral", 33, 5),
    ("QuantrupedMultiEnv_Centralized", 50, 4),
    ("QuantrupedMultiEnv_TwoSides", 20, 4),
    ("QuantrupedMultiEnv_SharedDecentralLegID", 24, 4),
    ("QuantrupedMultiEnv_SharedDecentralLegTransforms", 24, 4),
    ("QuantrupedMultiEnv_TwoDiags", 21, 4),
    ("QuantrupedMultiEnv_SingleNeighbor", 18, 4),
    ("QuantrupedMultiEnv_SingleDiagonal", 18, 4),
    ("QuantrupedMultiEnv_SingleToFront", 18, 4),
    ("QuantrupedMultiEnv_FullyDecentralGlobalCost", 22, 4),
    ("QuantrupedMultiEnv_Centralized", 1, 200),   # C1: one env, a full 200-step fragment
]


@pytest.mark.parametrize("env,n,T", ROLLOUT_ENVS)
def test_rollout_gae_parity(env, n, T):
    _rollout_gae_parity(env, n, T, None)


@pytest.mark.parametrize("env,n,T", [("QuantrupedMultiEnv_FullyDecentral", 24, 4),
                                     ("QuantrupedMultiEnv_Local", 20, 3),
                                     ("QuantrupedMultiEnv_Centralized", 16, 3)])
def test_rollout_gae_parity_target_velocity(env, n, T):
    """TVel variants (quantruped_v3.py:351-399): the 44th observation column
    (body_target_x_vel) is routed to every policy's input."""
    _rollout_gae_parity(env, n, T, {"env_config": {"target_velocity": [1.0]}})


@pytest.mark.parametrize("env,n,T", [("QuantrupedMultiEnv_FullyDecentral", 24, 5),
                                     ("QuantrupedMultiEnv_Local", 19, 4)])
def test_rollout_gae_parity_norm_reward(env, n, T):
    """norm_reward (quantruped_adaptor_multi_environment.py:173-186, DDRL_REWARD_NORM): every
    leg gets the whole forward reward minus n_agents x its own control + contact cost."""
    _rollout_gae_parity(env, n, T, {"env_config": {"norm_reward": True}})


def _rollout_gae_parity(env, n, T, config):
    ctx, cfg, inst = make_ctx(env, n, T, config)
    if config and config.get("env_config", {}).get("norm_reward"):
        assert cfg.reward_mode == N.REWARD_NORM and inst.reward_mode == "norm"
    rng = np.random.default_rng(11)
    params = init_params(ctx, cfg, 3)
    orc, norms, a_gpu, a_orc = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    _close(a_gpu, a_orc, msg="env actions")
    fn, fM, fS = ctx.filter_get()
    assert fn == orc.rs.n
    _close(fM, orc.rs.M, rtol=1e-12, atol=1e-12)
    _close(fS, orc.rs.S, rtol=1e-10, atol=1e-9)
    for p in range(cfg.n_policies):
        lay = ctx.layout[p]
        got = ctx.records_get(p)
        ref = orc.flat_records(p, lay)
        d, A = cfg.obs_dim[p], cfg.act_dim
        for name, sl in [("obs", slice(lay["obs"], lay["obs"] + d)),
                         ("act", slice(lay["act"], lay["act"] + A)),
                         ("logits", slice(lay["logit"], lay["logit"] + 2 * A)),
                         ("logp", lay["logp"]), ("vf", lay["vf"]), ("rew", lay["rew"]),
                         ("adv", lay["adv"]), ("vt", lay["vt"])]:
            _close(got[:, sl], ref[:, sl], rtol=1e-5, atol=2e-5, msg=f"{env} p{p} {name}")
        _close(ctx.last_values_get(p), orc.last_v[p], msg="bootstrap V(s_T)")
        an = ctx.adv_norm_get(p)
        _close(an, np.array(norms[p], np.float32), rtol=1e-5, atol=1e-6, msg="adv mean/std")
    ctx.close()


@pytest.mark.parametrize("env,n,T", [("QuantrupedMultiEnv_Local", 40, 5),
                                     ("QuantrupedMultiEnv_SharedDecentral", 24, 4)])
def test_rollout_with_policy_mean_std_filter(env, n, T):
    """observation_filter = MeanStdFilter: RLlib's per-policy RunningStat (unclipped) on top of
    the env-side filter; batched Chan merges on the device vs per-row pushes in the oracle."""
    ctx, cfg, inst = make_ctx(env, n, T, {"observation_filter": "MeanStdFilter"})
    assert cfg.policy_filter == 1
    rng = np.random.default_rng(17)
    params = init_params(ctx, cfg, 4)
    orc, norms, a_gpu, a_orc = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    _close(a_gpu, a_orc, msg="env actions")
    for p in range(cfg.n_policies):
        pn, pM, pS = ctx.policy_filter_get(p)
        assert pn == orc.pf[p].n
        _close(pM, orc.pf[p].M, rtol=1e-10, atol=1e-10)
        _close(pS, orc.pf[p].S, rtol=1e-9, atol=1e-8)
        dn, dM, dS = ctx.policy_filter_get(p, delta=True)
        assert dn == pn   # no sync yet: the delta is everything pushed
        lay = ctx.layout[p]
        got, ref = ctx.records_get(p), orc.flat_records(p, lay)
        d, A = cfg.obs_dim[p], cfg.act_dim
        _close(got[:, :d], ref[:, :d], rtol=1e-5, atol=2e-5, msg="filtered obs")
        _close(got[:, lay["logit"]:lay["logit"] + 2 * A], ref[:, lay["logit"]:lay["logit"] + 2 * A],
               rtol=1e-5, atol=2e-5, msg="logits")
    # set / get round trip recomputes the normalization constants
    pn, pM, pS = ctx.policy_filter_get(0)
    ctx.policy_filter_set(0, pn, pM * 0.5, pS)
    n2, M2, _ = ctx.policy_filter_get(0)
    assert n2 == pn and np.array_equal(M2, pM * 0.5)
    ctx.close()


def _batch_from_records(rec, lay, d, A, adv_norm):
    mean, den = adv_norm
    return dict(obs=rec[:, lay["obs"]:lay["obs"] + d], actions=rec[:, lay["act"]:lay["act"] + A],
                logits=rec[:, lay["logit"]:lay["logit"] + 2 * A], logp=rec[:, lay["logp"]],
                vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                vt=rec[:, lay["vt"]])


def _params_close(got, ref, lr, steps, msg):
    diff = np.abs(got - ref)
    frac = np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref))
    assert frac >= 0.999, f"{msg}: only {frac:.5f} of params within 1e-5 (max {diff.max():.3g})"
    assert diff.max() <= 2 * lr * steps + 1e-5, f"{msg}: max deviation {diff.max():.3g}"


TVEL = {"env_config": {"target_velocity": [1.0]}}   # obs 44: body_target_x_vel appended


UPDATE_CASES = [
    ("QuantrupedMultiEnv_Local", 64, 6, 3, None),
    ("QuantrupedMultiEnv_SharedDecentral", 32, 4, 2, None),
    ("QuantrupedMultiEnv_Centralized", 48, 8, 2, None),
    ("QuantrupedMultiEnv_SharedDecentralLegID", 32, 4, 2, None),
    ("QuantrupedMultiEnv_TwoSides", 33, 4, 2, None),             # A = 4, d = 27; ragged envs
    ("QuantrupedMultiEnv_TwoDiags", 35, 4, 2, None),             # A = 4, diagonal leg pairs
    ("QuantrupedMultiEnv_SingleNeighbor", 34, 4, 2, None),       # d = 27, 4 policies; R = 136
    ("QuantrupedMultiEnv_Centralized", 1, 160, 2, None),         # C1 shape: one env, A = 8, d = 43
    ("QuantrupedMultiEnv_FullyDecentral", 37, 5, 2, TVEL),        # d = 20 (TVel), 4 policies
    ("QuantrupedMultiEnv_Local", 40, 4, 2, TVEL),                 # d = 36 (TVel)
    ("QuantrupedMultiEnv_Centralized", 1, 200, 2, TVEL),         # C1 TVel: d = 44, A = 8, stride 76
]


@pytest.mark.parametrize("env,n,T,steps,config", UPDATE_CASES)
def test_ppo_update_parity(env, n, T, steps, config):
    import torch
    ctx, cfg, inst = make_ctx(env, n, T, config)
    rng = np.random.default_rng(5)
    params = init_params(ctx, cfg, 7, head_scale=1.0)
    orc, norms, _, _ = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    shuffles, perms, kls = [], [], []
    for p in range(cfg.n_policies):
        lay = ctx.layout[p]
        # feed the ORACLE's batch so the update parity does not inherit rollout rounding
        ctx.records_set(p, orc.flat_records(p, lay))
        ctx.adv_norm_set(p, *norms[p])
        R = T * lay["C"]
        sh, pe = O.sgd_schedule(np.random.default_rng(100 + p), R, 128, cfg.num_sgd_iter)
        shuffles.append(sh)
        perms.append(pe)
        kls.append(0.2 + 0.1 * p)
    dsh = [torch.from_numpy(s).cuda() for s in shuffles]
    dpe = [torch.from_numpy(s).cuda() for s in perms]
    ctx.ppo_update((1 << cfg.n_policies) - 1, dsh, dpe, kls, max_steps=steps)
    ctx.synchronize()
    for p in range(cfg.n_policies):
        lay = ctx.layout[p]
        d, A = cfg.obs_dim[p], cfg.act_dim
        batch = _batch_from_records(orc.flat_records(p, lay), lay, d, A, norms[p])
        shapes = O.ffn_param_shapes(d, 2 * A)
        adam = O.Adam(sum(int(np.prod(s)) for _, s in shapes), lr=cfg.lr)
        new, stats = O.ppo_update("ffn", params[p], shapes, adam, batch, shuffles[p], perms[p],
                                  np.float32(kls[p]), {"entropy_coeff": 0.0}, steps=steps)
        got = ctx.params_get(p)
        _params_close(got, O.pack(new, shapes), cfg.lr, steps, f"{env} p{p}")
        strict_params_check(got, "ffn", params[p], shapes, batch, shuffles[p], perms[p], kls[p], steps,
                            lr=cfg.lr, msg=f"{env} p{p}")
        m, v, b1p, b2p = ctx.adam_get(p)
        assert b1p == np.float32(adam.b1p) and b2p == np.float32(adam.b2p)
        st = ctx.ppo_stats(p, steps)
        for k, s in enumerate(stats):
            ref = [s["total_loss"], s["policy_loss"], s["vf_loss"], s["kl"], s["entropy"],
                   s["vf_explained_var"], s["grad_gnorm"]]
            _close(st[k, :7], np.array(ref, np.float32), rtol=1e-4, atol=1e-5, msg=f"stats step {k}")
    ctx.close()


def test_full_schedule_runs_and_stays_close():
    """Whole schedule (10 epochs x nb minibatches) for the Local config."""
    import torch
    env, n, T = "QuantrupedMultiEnv_Local", 64, 4   # R = 256 rows, nb = 2, 20 steps
    ctx, cfg, inst = make_ctx(env, n, T)
    rng = np.random.default_rng(9)
    params = init_params(ctx, cfg, 2, head_scale=1.0)
    orc, norms, _, _ = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    sh, pe = O.sgd_schedule(np.random.default_rng(1), T * n, 128, 10)
    for p in range(4):
        ctx.records_set(p, orc.flat_records(p, ctx.layout[p]))
        ctx.adv_norm_set(p, *norms[p])
    dsh = [torch.from_numpy(sh).cuda()] * 4
    dpe = [torch.from_numpy(pe).cuda()] * 4
    ctx.ppo_update(0xF, dsh, dpe, [0.2] * 4)
    ctx.synchronize()
    p = 1
    lay = ctx.layout[p]
    batch = _batch_from_records(orc.flat_records(p, lay), lay, 35, 2, norms[p])
    shapes = O.ffn_param_shapes(35, 4)
    adam = O.Adam(sum(int(np.prod(s)) for _, s in shapes))
    new, stats = O.ppo_update("ffn", params[p], shapes, adam, batch, sh, pe, np.float32(0.2), {})
    got = ctx.params_get(p)
    ref = O.pack(new, shapes)
    assert np.abs(got - ref).max() <= 1e-5
    strict_params_check(got, "ffn", params[p], shapes, batch, sh, pe, 0.2, 20, msg="full schedule")
    st = ctx.ppo_stats(p, 20)
    _close(st[-1, 0], stats[-1]["total_loss"], rtol=1e-3, atol=1e-4)
    # the last epoch's rows alone (what update_kl reads) are the same rows of the full read
    np.testing.assert_array_equal(ctx.ppo_stats(p, 2, first=18), st[18:])
    with pytest.raises(N.DdrlError):
        ctx.ppo_stats(p, 3, first=18)              # past the 10 x 2 schedule
    ctx.close()


def test_ddp_grad_and_apply_match_fused_step():
    """Gradient of two 64-row halves summed == 128-row gradient; apply == fused step."""
    import torch
    env, n, T = "QuantrupedMultiEnv_SharedDecentral", 32, 4
    ctx, cfg, inst = make_ctx(env, n, T)
    rng = np.random.default_rng(4)
    params = init_params(ctx, cfg, 8, head_scale=1.0)
    orc, norms, _, _ = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    lay = ctx.layout[0]
    ctx.records_set(0, orc.flat_records(0, lay))
    ctx.adv_norm_set(0, *norms[0])
    rows = np.random.default_rng(3).permutation(T * lay["C"])[:128].astype(np.int32)
    npar = ctx.n_params[0]
    g_full = torch.zeros(npar, device="cuda")
    g_a = torch.zeros(npar, device="cuda")
    g_b = torch.zeros(npar, device="cuda")
    r_all = torch.from_numpy(rows).cuda()
    ctx.ppo_grad(0, r_all, 128, 0.2, g_full)
    ctx.ppo_grad(0, r_all[:64].contiguous(), 64, 0.2, g_a)
    ctx.ppo_grad(0, r_all[64:].contiguous(), 64, 0.2, g_b)
    ctx.synchronize()
    gf = g_full.cpu().numpy()
    gs = (g_a + g_b).cpu().numpy()
    np.testing.assert_allclose(gs, gf, rtol=1e-4, atol=1e-6 * np.abs(gf).max())
    # oracle gradient of the same rows
    batch = _batch_from_records(orc.flat_records(0, lay), lay, 19, 2, norms[0])
    sl = {k: v[rows] for k, v in batch.items()}
    logits, value, cache = O.ffn_forward(params[0], sl["obs"])
    dl, dv, _ = O.ppo_loss_rows(logits, value, sl["actions"], sl["logits"], sl["logp"],
                                sl["vf_preds"], sl["adv"], sl["vt"], np.float32(0.2))
    shapes = O.ffn_param_shapes(19, 4)
    gref = O.pack(O.ffn_backward(params[0], cache, dl, dv), shapes)
    np.testing.assert_allclose(gf, gref, rtol=1e-4, atol=2e-5 * np.abs(gref).max())
    ctx.ppo_apply(0, g_full)
    ctx.synchronize()
    adam = O.Adam(npar)
    clipped, _ = O.clip_by_global_norm([gref], 0.5)
    ref = adam.apply(O.pack(params[0], shapes), clipped[0])
    _params_close(ctx.params_get(0), ref, 3e-4, 1, "ddp apply")
    # the same step as a one-step schedule whose first minibatch is `rows`, against fp64
    rest = np.setdiff1d(np.arange(T * lay["C"], dtype=np.int32), rows)
    sh1 = np.concatenate([rows, rest]).astype(np.int32)
    pe1 = np.arange(sh1.size // 128, dtype=np.int32)[None]
    strict_params_check(ctx.params_get(0), "ffn", params[0], shapes, batch, sh1, pe1, 0.2, 1, msg="ddp apply")
    ctx.close()


def test_policy_forward_matches_oracle():
    import torch
    ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_Local", 8, 2)
    params = init_params(ctx, cfg, 21)
    x = np.random.default_rng(0).normal(size=(203, 35)).astype(np.float32)
    logits = torch.zeros((203, 4), device="cuda")
    values = torch.zeros(203, device="cuda")
    ctx.policy_forward(2, torch.from_numpy(x).cuda(), 203, logits, values)
    ctx.synchronize()
    lr, vr, _ = O.ffn_forward(params[2], x)
    _close(logits.cpu().numpy(), lr)
    _close(values.cpu().numpy(), vr)
    ctx.close()


def test_host_buffer_loop_matches_device_loop():
    """ddrl_step_host / ddrl_act_host / ddrl_env_step_host (pinned host buffers, the host-env
    plane's interface) produce bit-identical records and actions to the device-buffer calls."""
    import torch
    from tests.gpu_harness import synthetic_inputs
    env, n, T = "QuantrupedMultiEnv_Local", 48, 5
    ctx_d, cfg, inst = make_ctx(env, n, T)
    ctx_h, _, _ = make_ctx(env, n, T)
    rng = np.random.default_rng(12)
    filt = _filt(cfg.obs_full_dim, rng)
    for c in (ctx_d, ctx_h):
        init_params(c, cfg, 4)
        c.filter_set(*filt)
    obs, eps, fw, cfrc, done = synthetic_inputs(rng, cfg, T)
    pin = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory()
    obs_h, eps_h, fw_h, cfrc_h, done_h = map(pin, (obs, eps, fw, cfrc, done))
    act_h = torch.zeros((n, 8), dtype=torch.float32).pin_memory()
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    actions = torch.zeros((n, 8), dtype=torch.float32, device="cuda")
    ctx_d.observe(dev(obs[0]))
    for t in range(T):
        ctx_d.act(t, dev(eps[t]), actions)
        ctx_d.reward(t, dev(fw[t]), dev(cfrc[t]), actions, dev(done[t]))
        ctx_d.observe(dev(obs[t + 1]))
        if t == 0:
            ctx_h.step_host(0, obs_h[0], eps_h[0], act_h)
        else:
            ctx_h.act_host(t, eps_h[t], act_h)
        ctx_h.synchronize()                      # the host env needs the actions
        np.testing.assert_array_equal(act_h.numpy(), actions.cpu().numpy())
        ctx_h.env_step_host(t, fw_h[t], cfrc_h[t], done_h[t], obs_h[t + 1])
    for c in (ctx_d, ctx_h):
        c.bootstrap()
        c.gae()
    ctx_d.synchronize()
    ctx_h.synchronize()
    for p in range(cfg.n_policies):
        np.testing.assert_array_equal(ctx_h.records_get(p), ctx_d.records_get(p))
    ctx_d.close()
    ctx_h.close()


def test_rollout_fragment_matches_step_loop():
    """ddrl_rollout_fragment (T x act / reward / observe + bootstrap in one call) produces the
    same records, bootstrap values and filter state as the per-step calls."""
    import torch
    from tests.gpu_harness import synthetic_inputs
    env, n, T = "QuantrupedMultiEnv_FullyDecentral", 40, 6
    ctx_a, cfg, inst = make_ctx(env, n, T)
    ctx_b, _, _ = make_ctx(env, n, T)
    rng = np.random.default_rng(21)
    filt = _filt(cfg.obs_full_dim, rng)
    for c in (ctx_a, ctx_b):
        init_params(c, cfg, 5)
        c.filter_set(*filt)
    obs, eps, fw, cfrc, done = synthetic_inputs(rng, cfg, T)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    obs_d, eps_d, fw_d, cfrc_d, done_d = map(dev, (obs, eps, fw, cfrc, done))
    act_a = torch.zeros((n, 8), dtype=torch.float32, device="cuda")
    act_b = torch.zeros((n, 8), dtype=torch.float32, device="cuda")
    ctx_a.observe(obs_d[0])
    for t in range(T):
        ctx_a.act(t, eps_d[t], act_a)
        ctx_a.reward(t, fw_d[t], cfrc_d[t], act_a, done_d[t])
        ctx_a.observe(obs_d[t + 1])
    ctx_a.bootstrap()
    ctx_b.observe(obs_d[0])
    ctx_b.rollout_fragment(obs_d, eps_d, fw_d, cfrc_d, done_d, act_b)
    ctx_a.synchronize()
    ctx_b.synchronize()
    for p in range(cfg.n_policies):
        np.testing.assert_array_equal(ctx_b.records_get(p), ctx_a.records_get(p))
        np.testing.assert_array_equal(ctx_b.last_values_get(p), ctx_a.last_values_get(p))
    fa, fb = ctx_a.filter_get(), ctx_b.filter_get()
    assert fa[0] == fb[0] and np.array_equal(fa[1], fb[1]) and np.array_equal(fa[2], fb[2])
    ctx_a.close()
    ctx_b.close()


def test_update_rejects_batch_smaller_than_a_minibatch():
    """A policy whose train batch (frag_len x agents) holds fewer rows than
    sgd_minibatch_size has no full minibatch: the update refuses it instead of reading past
    the shuffle (30 envs x T 4 = 120 rows per leg policy)."""
    import torch
    from ddrl_amd.native import DdrlError
    ctx, cfg, _ = make_ctx("QuantrupedMultiEnv_SingleNeighbor", 30, 4)
    sh = [torch.zeros(120, dtype=torch.int32, device="cuda") for _ in range(4)]
    pe = [torch.zeros((cfg.num_sgd_iter, 1), dtype=torch.int32, device="cuda") for _ in range(4)]
    with pytest.raises(DdrlError, match="fewer than one minibatch"):
        ctx.ppo_update(0xF, sh, pe, [0.2] * 4)
    ctx.close()
