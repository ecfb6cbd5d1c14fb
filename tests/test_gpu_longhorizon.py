"""Long-horizon update parity on the bench's own configuration.

BASELINE C2/C3 workload: QuantrupedMultiEnv_Local, 4096 envs x T = 200 -> R = 819,200 rows per
policy, nb = 6,400 minibatches per epoch.  The fused update launch runs all four policies as
the bench does (mask 0xF) and policy 0 is compared with the oracle over the same shuffle /
permutation (train_experiment_1_architecture_on_flat.py:116,133-134) after
H = 10, 100, 400, 1600, 3200 and 6400 sequential SGD steps (6400 = one full epoch).

Drift bound, a function of H derived from measured fp32 rounding.  Two fp32 implementations of
one H-step recursion do not agree to the last bit: every step's rounding feeds the next.  Each
horizon is measured against the fp64 trajectory of the same algorithm (oracle.with_dtype):
  * deterministic regime, H <= 1600: e32(H) = max |theta_numpy_fp32 - theta_fp64| is what fp32
    rounding alone costs; the HIP parameters must satisfy max |theta_HIP - theta_fp64| <=
    4 e32(H) + 2e-7 (the hardware tanh / exp / rcp / sqrt approximations, |err| ~1.5e-7, are
    per-step noise of the order of numpy's correctly rounded functions), every parameter
    within 1e-5 of fp64 (north_star) and within 1e-6 of numpy fp32, and every per-step learner
    statistic within 1e-4 relative (+1e-6 absolute) of fp64.  Measured (MI355X, r02): e32 / HIP
    6.9e-8 / 1.6e-7 (H = 10), 1.6e-7 / 1.8e-7 (100), 3.7e-6 / 4.1e-6 (400), 4.1e-6 / 4.5e-6 (1600).
  * after the bifurcation (between 1,600 and 3,200 steps a minibatch row's ratio / value clip
    switches branch in fp32 but not in fp64: every fp32 trajectory leaves the fp64 one by
    ~1e-2 and only ~1 % of parameters stay within 1e-5 -- numpy and HIP alike, and they stay
    within 5.4e-7 of each other at 3200), no fp32 implementation meets an absolute bar.  The
    bar is the spread of fp32 trajectories: seven more numpy fp32 runs that sum each
    minibatch's rows in a different (fixed, permuted) order -- the same mathematics, other
    roundings -- give s(H) = max over the eight numpy runs of the distance to fp64, for the
    parameters, the trained policy's outputs on 4,096 sampled rows, and the epoch means of the
    learner statistics (what update_kl consumes); HIP must be within 2 s(H) (+2e-7).  (r03:
    with four runs the sample of the spread was small enough that a HIP build whose head
    gradient sums its rows in the MFMA order landed at 2.03 s(H) on one statistic, the epoch
    mean policy loss; eight runs estimate the same spread from twice the sample.)
  * frozen ratios (round 4): the 2 s(H) bar alone would absorb a kernel change
    that walks a statistic toward its edge.  The HIP / spread ratio of every post-bifurcation
    quantity is printed and must stay within RATIO_MARGIN of its r03 value (R03_RATIO, measured
    on MI355X with the eight-run spread, profiles/r03/gpu_tests.log:118-127) as well as under 2.
"""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import init_params, make_ctx

pytestmark = pytest.mark.gpu
N_ENVS, T = 4096, 200
HORIZONS = [10, 100, 400, 1600, 3200, 6400]
ABS_BAR_UNTIL = 1600
STAT_KEYS = [(1, "policy_loss"), (2, "vf_loss"), (3, "kl"), (4, "entropy"), (6, "grad_gnorm")]
# HIP distance to fp64 / fp32 spread, r03 kernel (profiles/r03/gpu_tests.log:118-127)
R03_RATIO = {"theta@3200": 1.00, "theta@6400": 0.89, "logits": 0.93, "value": 1.10, "policy_loss": 0.33,
             "vf_loss": 0.95, "kl": 0.67, "entropy": 0.67, "grad_gnorm": 1.55}
RATIO_MARGIN = 0.25


def _check_ratio(name, dist, spread, ratios):
    """Record dist / spread and hold it to the r03 value + RATIO_MARGIN (and to the 2x bar)."""
    r = dist / spread if spread > 0 else (0.0 if dist == 0 else np.inf)
    ratios[name] = r
    assert r <= min(2.0, R03_RATIO[name] + RATIO_MARGIN) or dist <= 2e-7, \
        (name, f"HIP/spread {r:.3f} > r03 {R03_RATIO[name]:.2f} + {RATIO_MARGIN}")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _batch(rec, lay, d, A, norm):
    mean, den = norm
    return dict(obs=rec[:, lay["obs"]:lay["obs"] + d], actions=rec[:, lay["act"]:lay["act"] + A],
                logits=rec[:, lay["logit"]:lay["logit"] + 2 * A], logp=rec[:, lay["logp"]],
                vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                vt=rec[:, lay["vt"]])


def _row_order_variant(shuffle, seed):
    """The same minibatches with their 128 rows in another order (fp32 sums reassociated)."""
    order = np.random.default_rng(seed).permutation(128)
    nb = shuffle.size // 128
    out = shuffle.copy()
    out[:nb * 128] = shuffle[:nb * 128].reshape(nb, 128)[:, order].reshape(-1)
    return out


def _run(mod, params, shapes, batch, sh, pe, horizons):
    n = sum(int(np.prod(s)) for _, s in shapes)
    snaps = {h: None for h in horizons}
    _, stats = mod.ppo_update("ffn", params, shapes, mod.Adam(n), batch, sh, pe, 0.2, {}, steps=max(horizons),
                              snapshots=snaps)
    return {h: np.asarray(v, np.float64) for h, v in snaps.items()}, stats


@pytest.fixture(scope="module")
def local():
    import torch
    from ddrl_amd.synthetic import SyntheticRollout
    ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_Local", N_ENVS, T)
    params = init_params(ctx, cfg, 21, head_scale=1.0)     # the reference's 0.01 head init
    syn = SyntheticRollout(N_ENVS, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=3)
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, syn.dones_for_fragment(), syn.actions)
    ctx.gae()
    ctx.synchronize()
    del syn
    R = T * ctx.layout[0]["C"]
    assert R == 819200
    sched = [O.sgd_schedule(np.random.default_rng(40 + p), R, 128, 10) for p in range(4)]
    p, d, A = 0, cfg.obs_dim[0], cfg.act_dim
    batch = _batch(ctx.records_get(p), ctx.layout[p], d, A, ctx.adv_norm_get(p))
    yield ctx, cfg, params, sched, batch
    ctx.close()


def test_one_epoch_local_fullsize_against_fp64_trajectory(local):
    import torch
    ctx, cfg, params, sched, batch = local
    R = T * ctx.layout[0]["C"]
    dsh = [torch.from_numpy(s).cuda() for s, _ in sched]
    dpe = [torch.from_numpy(q).cuda() for _, q in sched]
    p, d, A = 0, cfg.obs_dim[0], cfg.act_dim
    shapes = O.ffn_param_shapes(d, 2 * A)
    sh, pe = sched[p]
    O64 = O.with_dtype(np.float64)
    th64, st64 = _run(O64, {k: v.astype(np.float64) for k, v in params[p].items()}, shapes, batch, sh, pe, HORIZONS)
    late = [h for h in HORIZONS if h > ABS_BAR_UNTIL]
    runs32 = [_run(O, params[p], shapes, batch, sh, pe, HORIZONS)]
    runs32 += [_run(O, params[p], shapes, batch, _row_order_variant(sh, 90 + k), pe, late) for k in range(7)]
    theta0 = [ctx.params_get(q) for q in range(4)]
    ratios = {}
    for H in HORIZONS:
        for q in range(4):      # same start for every horizon (the schedule restarts at step 0)
            ctx.params_set(q, theta0[q])
            ctx.adam_set(q, np.zeros(theta0[q].size), np.zeros(theta0[q].size), 0.9, 0.999)
        ctx.ppo_update(0xF, dsh, dpe, [0.2] * 4, max_steps=H)
        ctx.synchronize()
        got = ctx.params_get(p).astype(np.float64)
        egpu = np.abs(got - th64[H]).max()
        e32s = [np.abs(r[0][H] - th64[H]).max() for r in runs32 if H in r[0]]
        d32 = np.abs(got - runs32[0][0][H]).max()
        print(f"\nH={H}: max dev from fp64: numpy fp32 runs {[f'{e:.3g}' for e in e32s]}, HIP {egpu:.3g} "
              f"({np.mean(np.abs(got - th64[H]) <= 1e-5):.4f} within 1e-5); max |HIP - numpy fp32| {d32:.3g}",
              flush=True)
        st = ctx.ppo_stats(p, H).astype(np.float64)
        if H <= ABS_BAR_UNTIL:
            assert egpu <= 4 * e32s[0] + 2e-7, (H, egpu, e32s)
            assert egpu <= 1e-5 and d32 <= 1e-6, (H, egpu, d32)
            for col, k in STAT_KEYS:
                ref = np.array([s[k] for s in st64[:H]])
                dev = np.abs(st[:, col] - ref)
                assert np.all(dev <= 1e-4 * np.abs(ref) + 1e-6), (H, k, dev.max())
        else:
            assert egpu <= 2 * max(e32s) + 2e-7, (H, egpu, e32s)
            _check_ratio(f"theta@{H}", egpu, max(e32s), ratios)
    # H = 6400: the trained policy's outputs and the epoch-mean statistics against the spread
    assert np.abs(th64[6400] - O.pack(params[p], shapes)).max() > 0.1       # the policy did train
    rows = np.random.default_rng(1).choice(R, 4096, replace=False)
    x = torch.from_numpy(np.ascontiguousarray(batch["obs"][rows])).cuda()
    lg = torch.zeros((4096, 2 * A), device="cuda")
    vv = torch.zeros(4096, device="cuda")
    ctx.policy_forward(p, x, 4096, lg, vv)
    ctx.synchronize()
    out64 = O64.ffn_forward(O64.unpack(th64[6400], shapes), batch["obs"][rows])[:2]
    outs32 = [O.ffn_forward(O.unpack(r[0][6400].astype(np.float32), shapes), batch["obs"][rows])[:2] for r in runs32]
    for i, (name, g) in enumerate((("logits", lg.cpu().numpy()), ("value", vv.cpu().numpy()))):
        dg = np.abs(g - out64[i]).max()
        spread = max(np.abs(o[i] - out64[i]).max() for o in outs32)
        print(f"{name} vs fp64: HIP {dg:.3g}, fp32 spread {spread:.3g}")
        assert dg <= 2 * spread + 2e-7, name
        _check_ratio(name, dg, spread, ratios)
    for col, k in STAT_KEYS:
        ref = np.mean([s[k] for s in st64])
        dg = abs(st[:, col].mean() - ref)
        spread = max(abs(np.mean([s[k] for s in r[1]]) - ref) for r in runs32)
        print(f"epoch mean {k}: |HIP - fp64| {dg:.3g}, fp32 spread {spread:.3g} (ref {ref:.4g})")
        assert dg <= 2 * spread + 2e-7 * abs(ref), k
        _check_ratio(k, dg, spread, ratios)
    print("HIP / fp32-spread ratios (r03 in parentheses): " +
          ", ".join(f"{k} {v:.3f} ({R03_RATIO[k]:.2f})" for k, v in ratios.items()), flush=True)


@pytest.mark.timeout(1200)
def test_one_epoch_local_against_tie_following_fp64(local):
    """Round 6: the whole epoch (6,400 steps) at the bench configuration, for all four policies of
    the bench's launch, against the fp64 trajectory that follows the kernel at clip near-ties.

    The bifurcation between 1,600 and 3,200 steps that the test above meets with the fp32 spread
    is a clip decision whose fp64 margin is below fp32 resolution (DESIGN.md section 4,
    "Near-ties").  tests/gpu_harness.tie_following_trajectory walks the HIP trajectory one step at
    a time (ddrl_ppo_update_from) beside the fp64 one and takes HIP's outcome at every decision it
    took the other way.  The numpy fp32 oracle is measured the same way -- its own lockstep
    against the fp64 trajectory that follows numpy's outcomes -- which gives e32(H), the rounding
    drift of an fp32 implementation with the bifurcations taken out.  Through 3,200 steps every
    step whose HIP gradient departs from fp64's by more than the search threshold must be explained
    by flipped decisions (late in the epoch both implementations drift smoothly, gradient
    differences of 2e-4 - 6e-4 that no flip explains, and those steps are counted and printed).
    Bar, per policy and horizon:
    |HIP - fp64 following HIP| <= 4 e32(H) + 2e-7; within 1e-5 absolute through H = 3,200 for every
    policy (the north_star tolerance); every step's learner statistics within 1e-4 relative
    (+1e-6) of the tie-following fp64 ones; and the one-step-at-a-time HIP walk bit-identical to
    the bench's single 4-policy launch at every horizon."""
    import torch
    from tests.gpu_harness import HipLockstep, NumpyLockstep, tie_following_trajectory
    ctx, cfg, params, sched, batch0 = local
    A = cfg.act_dim
    shapes = [O.ffn_param_shapes(cfg.obs_dim[q], 2 * A) for q in range(4)]
    theta0 = [O.pack(params[q], shapes[q]) for q in range(4)]
    refs = []
    for q in range(4):
        batch = batch0 if q == 0 else _batch(ctx.records_get(q), ctx.layout[q], cfg.obs_dim[q], A, ctx.adv_norm_get(q))
        sh, pe = sched[q]
        npl = NumpyLockstep(params[q], shapes[q], batch, sh, pe, 0.2)
        missed32, missed = [], []
        tf32, _, ties32 = tie_following_trajectory(None, q, params[q], shapes[q], batch, sh, pe, 0.2, max(HORIZONS),
                                                   HORIZONS, impl=npl, missed=missed32)
        for r in range(4):
            ctx.params_set(r, theta0[r])
        hip = HipLockstep(ctx, q, theta0[q], sh, pe, 0.2)
        tf, tst, ties = tie_following_trajectory(ctx, q, params[q], shapes[q], batch, sh, pe, 0.2, max(HORIZONS),
                                                 HORIZONS, impl=hip, missed=missed)
        print(f"\nLocal policy {q}: HIP took {len(ties)} clip decisions the other way from fp64: " +
              "; ".join(f"step {t[0]} {t[1]} row {t[2]} margin {t[3]:.3g}" for t in ties) +
              f"; numpy fp32 took {len(ties32)}: " +
              "; ".join(f"step {t[0]} {t[1]} row {t[2]} margin {t[3]:.3g}" for t in ties32) +
              f"; steps whose gradient difference no flip explains: HIP {len(missed)} (from step "
              f"{missed[0][0] if missed else '-'}, at most {max([m[1] for m in missed], default=0):.3g}), numpy "
              f"{len(missed32)} (from step {missed32[0][0] if missed32 else '-'}, at most "
              f"{max([m[1] for m in missed32], default=0):.3g})", flush=True)
        # every departure of HIP from fp64 through the absolute-bar range is a flipped clip decision
        assert all(m[0] >= 3200 for m in missed), (q, missed[:5])
        assert all(t[6] <= 0.5 * t[7] for t in ties), (q, "a tie whose outcome the HIP gradient does not decide")
        e32 = {H: np.abs(npl.snaps[H] - tf32[H]).max() for H in HORIZONS}
        refs.append((tf, tst, e32, hip.snaps))
    dsh = [torch.from_numpy(s_).cuda() for s_, _ in sched]
    dpe = [torch.from_numpy(q_).cuda() for _, q_ in sched]
    fails = []
    for H in HORIZONS:
        for q in range(4):
            ctx.params_set(q, theta0[q])
            ctx.adam_set(q, np.zeros(theta0[q].size), np.zeros(theta0[q].size), 0.9, 0.999)
        ctx.ppo_update(0xF, dsh, dpe, [0.2] * 4, max_steps=H)
        ctx.synchronize()
        line = []
        for q in range(4):
            tf, tst, e32, walk = refs[q]
            got = ctx.params_get(q).astype(np.float64)
            etf = np.abs(got - tf[H]).max()
            bar = 4 * e32[H] + 2e-7
            line.append(f"p{q} {etf:.3g} (numpy fp32 {e32[H]:.3g})")
            if not np.array_equal(got, walk[H]):
                fails.append((q, H, "step-at-a-time walk differs from the 4-policy launch"))
            if not (etf <= bar and (H > 3200 or etf <= 1e-5)):
                fails.append((q, H, etf, e32[H]))
            st = ctx.ppo_stats(q, H).astype(np.float64)
            for col, k in STAT_KEYS:
                ref = np.array([s_[k] for s_ in tst[:H]])
                dev = np.abs(st[:, col] - ref)
                if not np.all(dev <= 1e-4 * np.abs(ref) + 1e-6):
                    fails.append((q, f"{k}@{H}", float(dev.max())))
        print(f"H={H}: |HIP - fp64 following HIP| (|numpy fp32 - fp64 following numpy|): " + "; ".join(line),
              flush=True)
    assert not fails, fails
