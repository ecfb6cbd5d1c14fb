"""Full-size checks at the shared-policy bench configurations, through
size-independent properties, on the GPU:

  C4  QuantrupedMultiEnv_SharedDecentral, 4096 envs x T = 200: one fcnet policy ("policy_legs",
      quantruped_singleDecentralizedController_environments.py:21-48) trained on all four legs,
      3,276,800 records, 25,600 minibatches per epoch;
  C5  QuantrupedMultiEnv_DecentralShared_Graph + "gnn", 2048 envs x T = 200: one GraphNet leg
      policy (quantruped_GraphDecentralizedController_environments.py:192-245,
      models/graph_net.py:32-45), 1,638,400 records, 12,800 minibatches per epoch, every step
      through the one-launch GNN step (reduction + clip + Adam in the gradient launch's tail,
      records pre-gathered in 1,024-step chunks).

For both: sampled records against the oracle recomputed from the record itself (forward,
DiagGaussian logp; C5 also the node index and the ego-quaternion columns against the raw
observation), 64 whole GAE chains against the oracle's recursion, the standardization constants
against fp64 statistics of all advantages, and the first three fused steps against the fp64
trajectory (tests/gpu_harness.strict_params_check).

C4, one quarter epoch (6,400 steps, the horizon tests/test_gpu_longhorizon.py runs for Local):
the absolute bar at every horizon against the fp64 trajectory that follows the kernel at clip
near-ties (test_c4_quarter_epoch_against_tie_following_fp64 says why: the r05 departure at
H = 680 is one value-clip decision whose fp64 margin is 1.1e-7).

C5: the numpy GraphNet costs ~20 ms per step, so a whole-epoch oracle trajectory is out of
reach; instead (a) 100 steps against fp64 (tests/gpu_harness.drift_check: HIP <= 4 e32 + 2e-7,
within 1e-5 of numpy fp32), (b) a whole epoch (12,800 steps, 13 record chunks) at lr = 0, where
the weights stay fixed and every step's learner statistics are the loss of its own minibatch at
the initial weights -- 24 steps across the epoch, both sides of every tested chunk boundary,
against the oracle one by one, and the weights back bit for bit -- and (c) a whole epoch at the
configured lr whose first 100 steps' statistics equal (a)'s bit for bit (the step does not
depend on the launch length) and whose statistics stay finite.
"""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from ddrl_amd.spec import make_cfg
from tests.gpu_harness import GNN_ENV, drift_check, init_gnn_params, init_params, make_ctx, strict_params_check

pytestmark = pytest.mark.gpu
T = 200
C4_ENV, C4_N = "QuantrupedMultiEnv_SharedDecentral", 4096
C5_N = 2048
HORIZONS = [10, 100, 400, 1600, 3200, 6400]
STAT_KEYS = [(1, "policy_loss"), (2, "vf_loss"), (3, "kl"), (4, "entropy"), (6, "grad_gnorm")]
_C5_STATS100 = {}   # the learner statistics of test_c5_100_steps_against_fp64's launch


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


def _rollout(env, n, seed, gnn):
    from ddrl_amd.synthetic import SyntheticRollout
    ctx, cfg, inst = make_ctx(env, n, T)
    params = init_gnn_params(ctx, seed, head_scale=1.0) if gnn else init_params(ctx, cfg, seed, head_scale=1.0)[0]
    syn = SyntheticRollout(n, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=seed)
    done = syn.dones_for_fragment()
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, done, syn.actions)
    ctx.gae()
    ctx.synchronize()
    return ctx, cfg, params, done.cpu().numpy(), syn


@pytest.fixture(scope="module")
def c4():
    ctx, cfg, params, done, syn = _rollout(C4_ENV, C4_N, 13, False)
    del syn
    rec = ctx.records_get(0)
    yield ctx, cfg, params, done, rec
    ctx.close()


@pytest.fixture(scope="module")
def c5():
    ctx, cfg, params, done, syn = _rollout(GNN_ENV, C5_N, 17, True)
    obs = syn.obs.cpu().numpy()
    del syn
    rec = ctx.records_get(0)
    yield ctx, cfg, params, done, rec, obs
    ctx.close()


def _ffn_batch(rec, lay, d, A, norm):
    mean, den = norm
    return dict(obs=rec[:, :d], actions=rec[:, lay["act"]:lay["act"] + A],
                logits=rec[:, lay["logit"]:lay["logit"] + 2 * A], logp=rec[:, lay["logp"]],
                vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                vt=rec[:, lay["vt"]])


def _gnn_batch(rec, lay, norm):
    mean, den = norm
    return dict(X=rec[:, :92].reshape(-1, 4, 23), node_idx=rec[:, 92].astype(np.int64),
                actions=rec[:, lay["act"]:lay["act"] + 2], logits=rec[:, lay["logit"]:lay["logit"] + 4],
                logp=rec[:, lay["logp"]], vf_preds=rec[:, lay["vf"]],
                adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32), vt=rec[:, lay["vt"]])


def _schedule(R, seed, epochs=10):
    import torch
    g = torch.Generator().manual_seed(seed)
    nb = R // 128
    sh = torch.randperm(R, generator=g).to(torch.int32)
    pe = torch.stack([torch.randperm(nb, generator=g) for _ in range(epochs)]).to(torch.int32)
    return sh, pe


def _reset(ctx, theta0):
    n = theta0.size
    ctx.params_set(0, theta0)
    ctx.adam_set(0, np.zeros(n, np.float32), np.zeros(n, np.float32), 0.9, 0.999)


def _gae_and_standardization(ctx, cfg, rec, done, k):
    lay = ctx.layout[0]
    C = ctx.layout[0]["C"]
    r = rec.reshape(T, C, -1)
    last_v = ctx.last_values_get(0)
    chains = np.random.default_rng(1).choice(C, 64, replace=False)
    adv, vt = O.gae_fragment(r[:, chains, lay["rew"]], r[:, chains, lay["vf"]], done[:, chains // k].astype(bool),
                             last_v[chains], cfg.gamma, cfg.lambda_)
    np.testing.assert_allclose(r[:, chains, lay["adv"]], adv, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(r[:, chains, lay["vt"]], vt, rtol=1e-5, atol=2e-5)
    a = r[:, :, lay["adv"]].reshape(-1).astype(np.float64)
    np.testing.assert_allclose(ctx.adv_norm_get(0), [a.mean(), max(1e-4, a.std())], rtol=1e-5, atol=1e-6)


# ------------------------------------------------------------------------------------- C4
def test_c4_records_match_oracle_rows(c4):
    ctx, cfg, params, _, rec = c4
    lay, d, A = ctx.layout[0], cfg.obs_dim[0], cfg.act_dim
    assert rec.shape[0] == T * C4_N * 4 and np.isfinite(rec).all()
    r = rec[np.random.default_rng(0).choice(rec.shape[0], 512, replace=False)]
    logits, value, _ = O.ffn_forward(params, r[:, :d])
    np.testing.assert_allclose(r[:, lay["logit"]:lay["logit"] + 2 * A], logits, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(r[:, lay["vf"]], value, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(r[:, lay["logp"]], O.dg_logp(logits, r[:, lay["act"]:lay["act"] + A]),
                               rtol=1e-5, atol=2e-5)
    assert np.abs(r[:, :d]).max() <= 10.0


def test_c4_gae_chains_and_standardization(c4):
    ctx, cfg, _, done, rec = c4
    _gae_and_standardization(ctx, cfg, rec, done, 4)


def test_c4_first_steps_against_fp64(c4):
    ctx, cfg, params, _, rec = c4
    shapes = O.ffn_param_shapes(cfg.obs_dim[0], 2 * cfg.act_dim)
    theta0 = O.pack(params, shapes)
    _reset(ctx, theta0)
    sh, pe = _schedule(rec.shape[0], 5)
    ctx.ppo_update(1, [sh.cuda()], [pe.cuda()], [0.2], max_steps=3)
    ctx.synchronize()
    batch = _ffn_batch(rec, ctx.layout[0], cfg.obs_dim[0], cfg.act_dim, ctx.adv_norm_get(0))
    strict_params_check(ctx.params_get(0), "ffn", params, shapes, batch, sh.numpy(), pe.numpy(), 0.2, 3,
                        msg="C4 full size")


def _row_order_variant(shuffle, seed):
    order = np.random.default_rng(seed).permutation(128)
    nb = shuffle.size // 128
    out = shuffle.copy()
    out[:nb * 128] = shuffle[:nb * 128].reshape(nb, 128)[:, order].reshape(-1)
    return out


def _ulp_variant(params, seed):
    """The same weights, every entry moved by one ulp up or down (random sign)."""
    rng = np.random.default_rng(seed)
    out = {}
    for k, v in params.items():
        v = np.asarray(v, np.float32)
        up = rng.random(v.shape) < 0.5
        out[k] = np.where(up, np.nextafter(v, np.float32(np.inf)), np.nextafter(v, np.float32(-np.inf))).astype(np.float32)
    return out


def _fast_tanh_oracle():
    """The fp32 oracle with the kernels' tanh formula (common.h tanh_fast) in fp32 numpy."""
    mod = O.with_dtype(np.float32)
    f32 = np.float32

    def tanh(x):
        x = np.asarray(x, f32)
        e = np.exp2(np.abs(x) * f32(2.8853900817779268)).astype(f32)
        r = (f32(1.0) / (e + f32(1.0))).astype(f32)
        return np.copysign((f32(1.0) - f32(2.0) * r).astype(f32), x)

    class _NP:
        def __getattr__(self, k):
            return getattr(np, k)

    shim = _NP()
    shim.tanh = tanh
    mod.np = shim
    return mod


def _run(mod, params, shapes, batch, sh, pe, horizons):
    n = sum(int(np.prod(s)) for _, s in shapes)
    snaps = {h: None for h in horizons}
    _, stats = mod.ppo_update("ffn", params, shapes, mod.Adam(n), batch, sh, pe, 0.2, {}, steps=max(horizons),
                              snapshots=snaps)
    return {h: np.asarray(v, np.float64) for h, v in snaps.items()}, stats


@pytest.mark.timeout(600)
def test_c4_quarter_epoch_against_tie_following_fp64(c4):
    """the C4 departure at H = 680 is a value-clip near-tie.

    Diagnosed in round 6 (tools/r06_c4_diag*.py, profiles/r06/): the HIP trajectory left the
    fp64 one at step 679 because of one row (row 101 of that minibatch) whose |V - vf_old| is
    10 (1 + 1.1e-7) in fp64 -- 1.1e-6 beyond vf_clip, about one ulp of 10 -- so fp64 and numpy
    clip it (no value gradient) and the kernel, whose dot-product order rounds V the other way,
    does not.  Neither the LSB-tagged exchange (a DDRL_UPDATE_SPLIT=1 launch, which has none, and
    the one-rank pair path, which adds untouched partials, both reproduce or avoid the departure
    with the row split, not the tags) nor the hardware rcp / sqrt (the numpy ensemble with Adam's
    and the clip scale's rounding perturbed does not depart) is involved.

    So the bar is the fp64 trajectory that takes the kernel's outcome at every clip decision the
    kernel took the other way (tests/gpu_harness.tie_following_trajectory: HIP walks its own
    trajectory one step at a time beside fp64, and a step whose HIP gradient departs from fp64's
    is explained by the flipped decisions among the smallest-margin rows).  Against it the
    absolute bar holds at EVERY horizon through the quarter epoch (6,400 steps): within
    4 e32(H) + 2e-7 and 1e-5 of it, where e32(H) = the numpy fp32 run's distance from the plain
    fp64 trajectory, and every step's learner statistics within 1e-4 relative (+1e-6).  The
    decisions HIP took the other way from fp64 are printed with their margins (r06: 5, all with
    |margin| <= 1.9e-6).  The plain-fp64 distances and a four-run fp32
    ensemble are printed for context; the mean statistics' HIP / spread ratios use the
    tie-following trajectory (HIP's distance from the fp64 path of its own tie decisions over the
    ensemble's spread around plain fp64) and must stay below 1.5."""
    import torch
    from tests.gpu_harness import tie_following_trajectory
    ctx, cfg, params, _, rec = c4
    d, A = cfg.obs_dim[0], cfg.act_dim
    shapes = O.ffn_param_shapes(d, 2 * A)
    theta0 = O.pack(params, shapes)
    lay = ctx.layout[0]
    batch = _ffn_batch(rec, lay, d, A, ctx.adv_norm_get(0))
    R = rec.shape[0]
    sh, pe = O.sgd_schedule(np.random.default_rng(44), R, 128, 10)
    H_MAX = max(HORIZONS)
    O64 = O.with_dtype(np.float64)
    th64, st64 = _run(O64, {k: v.astype(np.float64) for k, v in params.items()}, shapes, batch, sh, pe, HORIZONS)
    runs32 = [_run(O, params, shapes, batch, sh, pe, HORIZONS),
              _run(O, params, shapes, batch, _row_order_variant(sh, 90), pe, HORIZONS),
              _run(O, _ulp_variant(params, 200), shapes, batch, sh, pe, HORIZONS),
              _run(_fast_tanh_oracle(), params, shapes, batch, sh, pe, HORIZONS)]
    missed = []
    tf, tst, ties = tie_following_trajectory(ctx, 0, params, shapes, batch, sh, pe, 0.2, H_MAX, HORIZONS,
                                             missed=missed)
    print(f"\nC4 tie-following fp64 trajectory: {len(ties)} clip decisions taken the other way by HIP; "
          f"{len(missed)} steps whose gradient difference no flip explains {missed[:5]}:")
    for k, kind, i, m, nat, hip, best, second in ties:
        print(f"  step {k}: {'value' if kind == 'vf' else 'surrogate'} clip of minibatch row {i}, fp64 margin "
              f"{m:.3g}, fp64 {'passes' if nat else 'clips'}, HIP {'passes' if hip else 'clips'} (HIP gradient vs "
              f"fp64 with HIP's outcome {best:.3g}, with fp64's {second:.3g})")
    fails = []
    # every departure of the HIP gradient from fp64 is a flipped decision, read unambiguously
    fails += [("unexplained step", m) for m in missed]
    for t in ties:
        if not t[6] <= 0.5 * t[7]:
            fails.append(("undecided tie", t))
    dsh, dpe = torch.from_numpy(sh).cuda(), torch.from_numpy(pe).cuda()
    st = None
    for H in HORIZONS:
        _reset(ctx, theta0)
        ctx.ppo_update(1, [dsh], [dpe], [0.2], max_steps=H)
        ctx.synchronize()
        got = ctx.params_get(0).astype(np.float64)
        e32 = np.abs(runs32[0][0][H] - th64[H]).max()
        etf = np.abs(got - tf[H]).max()
        e64 = np.abs(got - th64[H]).max()
        ens = [np.abs(r[0][H] - th64[H]).max() for r in runs32]
        print(f"C4 H={H}: HIP - tie-following fp64 {etf:.3g} (bar {4 * e32 + 2e-7:.3g}); HIP - plain fp64 {e64:.3g}; "
              f"fp32 runs - plain fp64 {[f'{e:.3g}' for e in ens]}", flush=True)
        if not (etf <= 4 * e32 + 2e-7 and etf <= 1e-5):
            fails.append((f"theta@{H}", etf, e32))
        st = ctx.ppo_stats(0, H).astype(np.float64)
        for col, k in STAT_KEYS:
            ref = np.array([s[k] for s in tst[:H]])
            dev = np.abs(st[:, col] - ref)
            if not np.all(dev <= 1e-4 * np.abs(ref) + 1e-6):
                j = int(np.argmax(dev - 1e-4 * np.abs(ref)))
                fails.append((f"{k}@{H}", j, st[j, col], ref[j]))
    ratios = {}
    for col, k in STAT_KEYS:   # mean statistics over the 6,400 steps
        ref64 = np.mean([s[k] for s in st64])
        reftf = np.mean([s[k] for s in tst])
        dg = abs(st[:, col].mean() - reftf)
        spread = max(abs(np.mean([s[k] for s in r[1]]) - ref64) for r in runs32)
        ratios[k] = dg / spread if spread > 0 else (0.0 if dg == 0 else np.inf)
        print(f"C4 mean {k} over {H_MAX} steps: |HIP - tie-following fp64| {dg:.3g}, |HIP - plain fp64| "
              f"{abs(st[:, col].mean() - ref64):.3g}, fp32 ensemble spread {spread:.3g} (ratio {ratios[k]:.3f})")
        if not (ratios[k] < 1.5 or dg <= 2e-7 * abs(reftf)):
            fails.append((f"mean {k} ratio", ratios[k]))
    assert not fails, fails


# ------------------------------------------------------------------------------------- C5
def test_c5_records_match_oracle_rows(c5):
    ctx, cfg, params, _, rec, obs = c5
    lay = ctx.layout[0]
    C = lay["C"]
    assert rec.shape[0] == T * C5_N * 4 and C == 4 * C5_N and np.isfinite(rec).all()
    rows = np.random.default_rng(0).choice(rec.shape[0], 512, replace=False)
    r = rec[rows]
    X, node = r[:, :92].reshape(-1, 4, 23), r[:, 92]
    t, c = rows // C, rows % C
    np.testing.assert_array_equal(node, (c % 4).astype(np.float32))   # the agent's own node
    logits, value, _ = O.gnn_forward(params, X, node.astype(np.int64))
    np.testing.assert_allclose(r[:, lay["logit"]:lay["logit"] + 4], logits, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(r[:, lay["vf"]], value, rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(r[:, lay["logp"]], O.dg_logp(logits, r[:, lay["act"]:lay["act"] + 2]),
                               rtol=1e-5, atol=2e-5)
    # node features: the env-side filter's output, clipped at +-10; the ego quaternion of node n
    # from the raw observation of the row's env and step (leg_encoding_ego)
    assert np.abs(X[:, :, :19]).max() <= 10.0
    for i in range(0, 512, 8):
        raw = obs[t[i], c[i] // 4].astype(np.float64)
        q = np.stack([O.leg_encoding_ego(O.LEG_ANGLES[n], raw) for n in range(4)])
        np.testing.assert_allclose(X[i, :, 19:], q, rtol=1e-5, atol=1e-6)
    # the four rows of an env at one step carry the same graph
    same = rec[(rows // 4) * 4 + np.arange(4)[:, None]][:, :, :92]
    assert np.array_equal(same[0], same[1]) and np.array_equal(same[0], same[3])


def test_c5_gae_chains_and_standardization(c5):
    ctx, cfg, _, done, rec, _ = c5
    _gae_and_standardization(ctx, cfg, rec, done, 4)


def test_c5_first_steps_against_fp64(c5):
    ctx, cfg, params, _, rec, _ = c5
    shapes = O.gnn_param_shapes(4)
    _reset(ctx, O.pack(params, shapes))
    sh, pe = _schedule(rec.shape[0], 6)
    ctx.ppo_update(1, [sh.cuda()], [pe.cuda()], [0.2], max_steps=3)
    ctx.synchronize()
    batch = _gnn_batch(rec, ctx.layout[0], ctx.adv_norm_get(0))
    strict_params_check(ctx.params_get(0), "gnn", params, shapes, batch, sh.numpy(), pe.numpy(), 0.2, 3,
                        msg="C5 full size")


@pytest.fixture(scope="module")
def c5_schedule(c5):
    return _schedule(c5[4].shape[0], 8)


def test_c5_100_steps_against_fp64(c5, c5_schedule):
    ctx, cfg, params, _, rec, _ = c5
    shapes = O.gnn_param_shapes(4)
    _reset(ctx, O.pack(params, shapes))
    sh, pe = c5_schedule
    ctx.ppo_update(1, [sh.cuda()], [pe.cuda()], [0.2], max_steps=100)
    ctx.synchronize()
    batch = _gnn_batch(rec, ctx.layout[0], ctx.adv_norm_get(0))
    drift_check(ctx.params_get(0), "gnn", params, shapes, batch, sh.numpy(), pe.numpy(), 0.2, 100)
    _C5_STATS100["st"] = ctx.ppo_stats(0, 100)


C5_HORIZONS = [10, 100, 400, 1000, 2000, 4000]


@pytest.mark.timeout(900)
def test_c5_4000_steps_against_tie_following_fp64(c5, c5_schedule):
    """Round 6: the one-launch GraphNet step over 4,000 sequential steps at full size (forty times
    test_c5_100_steps_against_fp64's horizon), against the fp64 trajectory that takes the kernel's
    outcome at clip near-ties (tests/gpu_harness.tie_following_trajectory, model "gnn"; DESIGN.md
    section 4 "Near-ties"): within 4 e32(H) + 2e-7 and 1e-5 at every horizon, e32 = the numpy
    fp32 run's distance from plain fp64, and every step's learner statistics within 1e-4
    relative (+1e-6).  The numpy GraphNet's cost per step sets the horizon; a whole epoch (12,800
    steps, 9.6e-6 at its end) was walked with tools/r06_long_walk.py (profiles/r06/long_walk_c5.log)."""
    import torch
    from tests.gpu_harness import tie_following_trajectory
    ctx, cfg, params, _, rec, _ = c5
    shapes = O.gnn_param_shapes(4)
    theta0 = O.pack(params, shapes)
    sh_t, pe_t = c5_schedule
    sh, pe = sh_t.numpy(), pe_t.numpy()
    batch = _gnn_batch(rec, ctx.layout[0], ctx.adv_norm_get(0))
    H_MAX = max(C5_HORIZONS)
    O64 = O.with_dtype(np.float64)
    n = theta0.size

    def run(mod, p):
        snaps = {h: None for h in C5_HORIZONS}
        mod.ppo_update("gnn", p, shapes, mod.Adam(n), batch, sh, pe, 0.2, {}, steps=H_MAX, snapshots=snaps)
        return {h: np.asarray(v, np.float64) for h, v in snaps.items()}

    th64 = run(O64, {k: v.astype(np.float64) for k, v in params.items()})
    th32 = run(O, params)
    missed = []
    tf, tst, ties = tie_following_trajectory(ctx, 0, params, shapes, batch, sh, pe, 0.2, H_MAX, C5_HORIZONS,
                                             model="gnn", missed=missed)
    print(f"\nC5: {len(ties)} clip decisions taken the other way by HIP: " +
          "; ".join(f"step {t[0]} {t[1]} row {t[2]} margin {t[3]:.3g}" for t in ties) +
          f"; {len(missed)} steps whose gradient difference no flip explains {missed[:5]}")
    assert not missed, missed[:5]
    assert all(t[6] <= 0.5 * t[7] for t in ties), "a tie whose outcome the HIP gradient does not decide"
    dsh, dpe = sh_t.cuda(), pe_t.cuda()
    fails = []
    for H in C5_HORIZONS:
        _reset(ctx, theta0)
        ctx.ppo_update(1, [dsh], [dpe], [0.2], max_steps=H)
        ctx.synchronize()
        got = ctx.params_get(0).astype(np.float64)
        e32 = np.abs(th32[H] - th64[H]).max()
        etf = np.abs(got - tf[H]).max()
        print(f"C5 H={H}: HIP - tie-following fp64 {etf:.3g} (bar {min(4 * e32 + 2e-7, 1e-5):.3g}); HIP - plain "
              f"fp64 {np.abs(got - th64[H]).max():.3g}; numpy fp32 - plain fp64 {e32:.3g}", flush=True)
        if not (etf <= 4 * e32 + 2e-7 and etf <= 1e-5):
            fails.append((H, etf, e32))
        st = ctx.ppo_stats(0, H).astype(np.float64)
        for col, k in STAT_KEYS:
            ref = np.array([s_[k] for s_ in tst[:H]])
            dev = np.abs(st[:, col] - ref)
            if not np.all(dev <= 1e-4 * np.abs(ref) + 1e-6):
                fails.append((f"{k}@{H}", float(dev.max())))
    assert not fails, fails


def test_c5_epoch_at_lr0_statistics_step_by_step(c5, c5_schedule):
    import torch
    from ddrl_amd import native as N
    ctx0, cfg0, params, _, rec, _ = c5
    cfg_lr0, _ = make_cfg(GNN_ENV, C5_N, T, {"lr": 0.0})
    ctx = N.Context(cfg_lr0, 0, torch.cuda.current_stream().cuda_stream)
    shapes = O.gnn_param_shapes(4)
    theta0 = O.pack(params, shapes)
    _reset(ctx, theta0)
    ctx.records_set(0, rec)
    norm = ctx0.adv_norm_get(0)
    ctx.adv_norm_set(0, *norm)
    sh, pe = c5_schedule
    nb = rec.shape[0] // 128
    assert nb == 12800
    ctx.ppo_update(1, [sh.cuda()], [pe.cuda()], [0.2], max_steps=nb)
    ctx.synchronize()
    np.testing.assert_array_equal(ctx.params_get(0), theta0)
    st = ctx.ppo_stats(0, nb)
    assert np.isfinite(st).all()
    batch = _gnn_batch(rec, ctx.layout[0], norm)
    picks = sorted(set([0, 1, 1023, 1024, 1025, 2047, 2048, 6143, 6144, 11263, 11264, 12287, 12288, 12799] +
                       list(np.random.default_rng(3).choice(nb, 10, replace=False))))
    for k in picks:
        _, stats = O.ppo_update("gnn", params, shapes, O.Adam(theta0.size, lr=0.0), batch, sh.numpy(),
                                pe.numpy()[:1, k:k + 1], np.float32(0.2), {"entropy_coeff": 0.0}, steps=1)
        s0 = stats[0]
        ref = [s0["total_loss"], s0["policy_loss"], s0["vf_loss"], s0["kl"], s0["entropy"], s0["vf_explained_var"],
               s0["grad_gnorm"]]
        # vf_explained_var = 1 - Var(vt - vf) / Var(vt) from fp32 moment sums (reported, not used by
        # the update): at this rollout's vf_loss ~180 its cancellation error reaches ~1e-5 (measured
        # 1.2e-5 at one step), so that column gets 1e-4 absolute
        np.testing.assert_allclose(st[k, [0, 1, 2, 3, 4, 6]], np.array(ref, np.float32)[[0, 1, 2, 3, 4, 6]],
                                   rtol=1e-4, atol=1e-5, err_msg=f"C5 lr=0 epoch, step {k}")
        assert abs(st[k, 5] - ref[5]) <= 1e-4, (k, st[k, 5], ref[5])
    ctx.close()


def test_c5_epoch_at_configured_lr(c5, c5_schedule):
    ctx, cfg, params, _, rec, _ = c5
    _reset(ctx, O.pack(params, O.gnn_param_shapes(4)))
    sh, pe = c5_schedule
    nb = rec.shape[0] // 128
    ctx.ppo_update(1, [sh.cuda()], [pe.cuda()], [0.2], max_steps=nb)
    ctx.synchronize()
    st = ctx.ppo_stats(0, nb)
    assert np.isfinite(st).all() and np.isfinite(ctx.params_get(0)).all()
    if "st" in _C5_STATS100:   # the 100-step launch of test_c5_100_steps_against_fp64
        np.testing.assert_array_equal(st[:100], _C5_STATS100["st"])
    print(f"\nC5 epoch means: policy_loss {st[:, 1].mean():.4g}, vf_loss {st[:, 2].mean():.4g}, "
          f"kl {st[:, 3].mean():.4g}, entropy {st[:, 4].mean():.4g}, grad_gnorm {st[:, 6].mean():.4g}")
