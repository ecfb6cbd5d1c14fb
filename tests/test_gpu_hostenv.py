"""f1 host env plane: the pipelined host rollout (ddrl_rollout_hostenv:
env groups stepped by the C++ thread pool into pinned buffers while the device runs the other
groups' reward / observe / act) against the synchronous device loop over the same ranged
calls (ddrl_observe_range / ddrl_act_range / ddrl_reward_range on device buffers, host env
stepped in between with full synchronization).  Same env seed, same noise, same weights and
filter: the records, filter statistics and bootstrap values must be bit-identical.

Oracle anchor: the device loop also captures the host env plane's own raw
outputs (reset observations, then per step fw / cfrc / done / observations), and the CPU oracle
(OracleRollout / GnnOracleRollout: filter, routing, forward, sampling, rewards, bootstrap, fp64
GAE) runs over exactly those arrays and the same noise; the records of both HIP paths must match
it within the rollout parity tolerance of test_gpu_parity.py (1e-5 relative + 2e-5 absolute),
the env-side filter statistics within 1e-12 / 1e-9."""
import numpy as np
import pytest

from ddrl_amd import native as N
from tests.gpu_harness import GnnOracleRollout, OracleRollout, init_params, make_ctx

pytestmark = pytest.mark.gpu


def _device_loop(ctx, cfg, env, eps, groups):
    import torch
    n, T, D = cfg.n_envs, cfg.frag_len, cfg.obs_full_dim
    lo = [n * k // groups for k in range(groups + 1)]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    env.reset()
    trace = [env.obs.copy()]
    obs = dev(env.obs)
    fw = torch.zeros(n, device="cuda")
    cfrc = torch.zeros((n, 14, 6), device="cuda")
    done = torch.zeros(n, dtype=torch.uint8, device="cuda")
    act = torch.zeros((n, 8), device="cuda")
    for k in range(groups):
        ctx.observe_range(obs, lo[k], lo[k + 1])
        ctx.act_range(0, lo[k], lo[k + 1], eps[0], act)
    for t in range(T):
        for k in range(groups):
            e0, e1 = lo[k], lo[k + 1]
            torch.cuda.synchronize()
            env.act[e0:e1] = act[e0:e1].cpu().numpy()
            env.step(e0, e1)
            fw[e0:e1] = dev(env.fw[e0:e1])
            cfrc[e0:e1] = dev(env.cfrc[e0:e1])
            done[e0:e1] = dev(env.done[e0:e1])
            obs[e0:e1] = dev(env.obs[e0:e1])
            if k == 0:
                trace.append([None] * 4)
            for j, a in enumerate((env.fw, env.cfrc, env.done, env.obs)):
                trace[-1][j] = a.copy() if k == 0 else trace[-1][j]
                trace[-1][j][e0:e1] = a[e0:e1]
            ctx.reward_range(t, e0, e1, fw, cfrc, act, done)
            ctx.observe_range(obs, e0, e1)
            if t + 1 < T:
                ctx.act_range(t + 1, e0, e1, eps[t + 1], act)
    ctx.bootstrap()
    ctx.synchronize()
    return trace


def _oracle_over_trace(cfg, inst, params, filt, trace, eps, gnn, groups):
    """The oracle rollout over the host env plane's raw outputs (see the module docstring).
    Both HIP paths observe each env group by its own ranged call (one filter push and
    normalization per group), so the oracle filters group by group too."""
    n = cfg.n_envs
    lo = [n * k // groups for k in range(groups + 1)]
    orc = (GnnOracleRollout if gnn else OracleRollout)(cfg, inst, params, filt)
    orc.observe(trace[0], lo)
    for t, (fw, cfrc, done, obs) in enumerate(trace[1:]):
        a = orc.act(t, eps[t])
        orc.reward(t, fw, cfrc, a, done)
        orc.observe(obs, lo)
    orc.bootstrap()
    return orc, orc.gae()


@pytest.mark.parametrize("env_name,n,T,groups,config", [
    ("QuantrupedMultiEnv_Local", 256, 24, 2, None),
    ("QuantrupedMultiEnv_Local", 203, 12, 3, {"observation_filter": "MeanStdFilter"}),   # ragged groups
    ("QuantrupedMultiEnv_Centralized", 64, 10, 2, None),
    ("QuantrupedMultiEnv_DecentralShared_Graph", 96, 10, 2, None),
    ("QuantrupedMultiEnv_FullyDecentral", 80, 10, 1, {"env_config": {"target_velocity": [1.0]}}),
    # a 2-velocity list, every env drawing its own on each reset
    ("QuantrupedMultiEnv_Local", 160, 16, 2, {"env_config": {"target_velocity": [0.5, 1.5]}}),
])
def test_pipelined_host_rollout_matches_device_loop(env_name, n, T, groups, config):
    import torch
    ctxs, envs = [], []
    for threads in (4, 1):
        ctx, cfg, inst = make_ctx(env_name, n, T, config)
        gnn = cfg.model_kind == N.MODEL_GNN
        if gnn:
            from tests.gpu_harness import init_gnn_params
            params = init_gnn_params(ctx, 5, head_scale=1.0)
        else:
            params = init_params(ctx, cfg, 5, head_scale=1.0)
        filt = (1000.0, np.linspace(-0.5, 0.5, cfg.obs_full_dim), np.full(cfg.obs_full_dim, 2000.0))
        ctx.filter_set(*filt)
        ctxs.append(ctx)
        tv = ((config or {}).get("env_config") or {}).get("target_velocity", [1.0])
        envs.append(N.HostEnv(n, cfg.obs_full_dim, threads, seed=11, target_velocity=tv))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    eps = torch.randn((T, n, cfg.n_agents, cfg.act_dim), device="cuda", generator=gen)
    ctxs[0].rollout_hostenv(envs[0], eps, groups=groups, reset=True)
    trace = _device_loop(ctxs[1], cfg, envs[1], eps, groups)
    for c in ctxs:
        c.gae()
        c.synchronize()
    for p in range(cfg.n_policies):
        a, b = ctxs[0].records_get(p), ctxs[1].records_get(p)
        assert np.isfinite(a).all()
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(ctxs[0].last_values_get(p), ctxs[1].last_values_get(p))
        np.testing.assert_array_equal(ctxs[0].adv_norm_get(p), ctxs[1].adv_norm_get(p))
    fa, fb = ctxs[0].filter_get(), ctxs[1].filter_get()
    assert fa[0] == fb[0] == 1000.0 + n * (T + 1)
    np.testing.assert_array_equal(fa[1], fb[1])
    np.testing.assert_array_equal(fa[2], fb[2])
    # the host envs themselves ended in the same state (thread count does not matter)
    np.testing.assert_array_equal(envs[0].obs, envs[1].obs)
    if cfg.obs_full_dim == 44:
        tvs = envs[0].target_velocities
        np.testing.assert_array_equal(tvs, envs[1].target_velocities)
        np.testing.assert_array_equal(envs[0].obs[:, 43], tvs)
        assert set(np.unique(tvs)) == set(np.float32(tv))   # both velocities in use
    # both against the oracle run on the host env plane's raw outputs
    assert len(trace) == T + 1
    orc, norms = _oracle_over_trace(cfg, inst, params, filt, trace, eps.cpu().numpy(), gnn, groups)
    assert fa[0] == orc.rs.n
    np.testing.assert_allclose(fa[1], orc.rs.M, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(fa[2], orc.rs.S, rtol=1e-10, atol=1e-9)
    for p in range(cfg.n_policies):
        lay = ctxs[0].layout[p]
        got, ref = ctxs[0].records_get(p), orc.flat_records(p, lay)
        d, A = (93 if gnn else cfg.obs_dim[p]), cfg.act_dim      # GNN rows: X (4 x 23) + node index
        for name, sl in [("obs", slice(lay["obs"], lay["obs"] + d)), ("act", slice(lay["act"], lay["act"] + A)),
                         ("logits", slice(lay["logit"], lay["logit"] + 2 * A)), ("logp", lay["logp"]),
                         ("vf", lay["vf"]), ("rew", lay["rew"]), ("adv", lay["adv"]), ("vt", lay["vt"])]:
            np.testing.assert_allclose(got[:, sl], ref[:, sl], rtol=1e-5, atol=2e-5,
                                       err_msg=f"{env_name} p{p} {name} vs oracle")
        np.testing.assert_allclose(ctxs[0].last_values_get(p), orc.last_v[p], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(ctxs[0].adv_norm_get(p), np.array(norms[p], np.float32), rtol=1e-5, atol=1e-6)
    for c in ctxs:
        c.close()
    for e in envs:
        e.close()


def test_ranged_calls_cover_the_whole_step():
    """One group = the whole shard: ranged observe / act / reward equal the plain calls."""
    import torch
    n, T = 100, 3
    ctxs = []
    for _ in range(2):
        ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_Local", n, T)
        init_params(ctx, cfg, 8, head_scale=1.0)
        ctxs.append(ctx)
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    obs = torch.randn((T + 1, n, 43), device="cuda", generator=g)
    eps = torch.randn((T, n, 4, 2), device="cuda", generator=g)
    fw = torch.randn((T, n), device="cuda", generator=g)
    cf = torch.randn((T, n, 14, 6), device="cuda", generator=g)
    act = [torch.zeros((n, 8), device="cuda") for _ in range(2)]
    ctxs[0].observe(obs[0])
    ctxs[1].observe_range(obs[0], 0, n)
    for t in range(T):
        ctxs[0].act(t, eps[t], act[0])
        ctxs[1].act_range(t, 0, n, eps[t], act[1])
        ctxs[0].reward(t, fw[t], cf[t], act[0])
        ctxs[1].reward_range(t, 0, n, fw[t], cf[t], act[1])
        ctxs[0].observe(obs[t + 1])
        ctxs[1].observe_range(obs[t + 1], 0, n)
    for c in ctxs:
        c.bootstrap()
        c.gae()
        c.synchronize()
    for p in range(4):
        np.testing.assert_array_equal(ctxs[0].records_get(p), ctxs[1].records_get(p))
    with pytest.raises(N.DdrlError):
        ctxs[0].act_range(0, 50, 50, eps[0], act[0])      # empty range is refused
    with pytest.raises(N.DdrlError):
        ctxs[0].observe_range(obs[0], 0, n + 1)          # past the shard
    for c in ctxs:
        c.close()
