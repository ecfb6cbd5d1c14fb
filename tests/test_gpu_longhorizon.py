"""Long-horizon update parity on the bench's own configuration.

BASELINE C2/C3 workload: QuantrupedMultiEnv_Local, 4096 envs x T = 200 -> R = 819,200 rows per
policy, nb = 6,400 minibatches per epoch.  The fused update launch runs all four policies as
the bench does (mask 0xF) and policy 0 is compared with the oracle over the same shuffle /
permutation (train_experiment_1_architecture_on_flat.py:116,133-134) at the
horizons H = 10, 100, 400, 1600, 3200 and 6400 sequential SGD steps (6400 = one full epoch).

Drift bound (a function of H, derived from measured fp32 rounding).  Two fp32 implementations
of the same H-step recursion do not agree to the last bit: every step's rounding feeds the
next.  Each horizon is therefore measured against the fp64 trajectory of the same algorithm
(oracle.with_dtype(np.float64)):
    e32(H)  = max |theta_numpy_fp32 - theta_fp64|   (what fp32 rounding alone costs)
    egpu(H) = max |theta_HIP - theta_fp64|
and every horizon requires egpu(H) <= 4 e32(H) + 2e-7 (the kernel's hardware tanh / exp / rcp /
sqrt approximations, |err| ~1.5e-7 each, are per-step noise of the order of numpy's correctly
rounded functions).  Measured on MI355X (r02): e32 / egpu = 6.9e-8 / 1.6e-7 (H = 10),
1.6e-7 / 1.8e-7 (100), 3.7e-6 / 4.1e-6 (400), 4.1e-6 / 4.5e-6 (1600); at 6400 the trajectory
itself bifurcates (a minibatch row's PPO ratio or value clip switches branch: the fp32
trajectories leave the fp64 one by ~2e-2 -- numpy 0.0205, HIP 0.015 -- and only 0.6 % of numpy's
parameters stay within 1e-5), so no fp32 implementation meets an absolute bar there.
Absolute bars where they are meaningful (H <= 1600, before the bifurcation): every parameter
within 1e-5 of fp64 (north_star) and within 1e-6 of numpy fp32; per-step learner statistics
within 1e-4 relative (+1e-6 absolute) of fp64.  At H = 6400 the trained policy's outputs on
4,096 sampled rows and the epoch-mean statistics (what update_kl consumes) must be no farther
from the fp64 trajectory than 4x numpy fp32's distance (+1e-6).
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


def test_one_epoch_local_fullsize_against_fp64_trajectory():
    import torch
    from ddrl_amd.synthetic import SyntheticRollout
    ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_Local", N_ENVS, T)
    params = init_params(ctx, cfg, 21, head_scale=1.0)     # the reference's 0.01 head init
    syn = SyntheticRollout(N_ENVS, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=3)
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, syn.dones_for_fragment(), syn.actions)
    ctx.gae()
    ctx.synchronize()
    R = T * ctx.layout[0]["C"]
    assert R == 819200
    sched = [O.sgd_schedule(np.random.default_rng(40 + p), R, 128, 10) for p in range(4)]
    dsh = [torch.from_numpy(s).cuda() for s, _ in sched]
    dpe = [torch.from_numpy(q).cuda() for _, q in sched]
    p, d, A = 0, cfg.obs_dim[0], cfg.act_dim
    lay = ctx.layout[p]
    batch = _batch(ctx.records_get(p), lay, d, A, ctx.adv_norm_get(p))
    shapes = O.ffn_param_shapes(d, 2 * A)
    n = sum(int(np.prod(s)) for _, s in shapes)
    sh, pe = sched[p]
    O64 = O.with_dtype(np.float64)
    p64 = {k: v.astype(np.float64) for k, v in params[p].items()}
    theta0 = [ctx.params_get(q) for q in range(4)]
    for H in HORIZONS:
        for q in range(4):      # same start for every horizon (the schedule restarts at step 0)
            ctx.params_set(q, theta0[q])
            ctx.adam_set(q, np.zeros(theta0[q].size), np.zeros(theta0[q].size), 0.9, 0.999)
        ctx.ppo_update(0xF, dsh, dpe, [0.2] * 4, max_steps=H)
        ctx.synchronize()
        got = ctx.params_get(p).astype(np.float64)
        new32, st32 = O.ppo_update("ffn", params[p], shapes, O.Adam(n), batch, sh, pe, 0.2, {}, steps=H)
        new64, st64 = O64.ppo_update("ffn", p64, shapes, O64.Adam(n), batch, sh, pe, 0.2, {}, steps=H)
        th32 = O.pack(new32, shapes).astype(np.float64)
        th64 = O64.pack(new64, shapes)
        e32, egpu, d32 = np.abs(th32 - th64).max(), np.abs(got - th64).max(), np.abs(got - th32).max()
        print(f"\nH={H}: max dev from fp64: numpy fp32 {e32:.3g} ({np.mean(np.abs(th32 - th64) <= 1e-5):.4f} "
              f"within 1e-5), HIP {egpu:.3g} ({np.mean(np.abs(got - th64) <= 1e-5):.4f}); "
              f"max |HIP - numpy fp32| {d32:.3g}", flush=True)
        assert egpu <= 4 * e32 + 2e-7, (H, egpu, e32)
        st = ctx.ppo_stats(p, H).astype(np.float64)
        if H <= ABS_BAR_UNTIL:
            assert egpu <= 1e-5 and d32 <= 1e-6, (H, egpu, d32)
            for col, k in STAT_KEYS:
                ref = np.array([s[k] for s in st64])
                dev = np.abs(st[:, col] - ref)
                print(f"  {k}: max |HIP - fp64| {dev.max():.3g} (|ref| median {np.median(np.abs(ref)):.3g})")
                assert np.all(dev <= 1e-4 * np.abs(ref) + 1e-6), (H, k)
    # H = 6400 (one epoch): outputs and epoch-mean statistics relative to numpy fp32's distance
    assert np.abs(th64 - O.pack(params[p], shapes)).max() > 0.1       # the policy did train
    rows = np.random.default_rng(1).choice(R, 4096, replace=False)
    x = torch.from_numpy(np.ascontiguousarray(batch["obs"][rows])).cuda()
    lg = torch.zeros((4096, 2 * A), device="cuda")
    vv = torch.zeros(4096, device="cuda")
    ctx.policy_forward(p, x, 4096, lg, vv)
    ctx.synchronize()
    l64, v64, _ = O64.ffn_forward(new64, batch["obs"][rows])
    l32, v32, _ = O.ffn_forward(new32, batch["obs"][rows])
    for name, g, r64, r32 in (("logits", lg.cpu().numpy(), l64, l32), ("value", vv.cpu().numpy(), v64, v32)):
        dg, dn = np.abs(g - r64).max(), np.abs(r32 - r64).max()
        print(f"{name} vs fp64: HIP {dg:.3g}, numpy fp32 {dn:.3g}")
        assert dg <= 4 * dn + 1e-6, name
    for col, k in STAT_KEYS:
        ref = np.mean([s[k] for s in st64])
        dg = abs(st[:, col].mean() - ref)
        dn = abs(np.mean([s[k] for s in st32]) - ref)
        print(f"epoch mean {k}: |HIP - fp64| {dg:.3g}, |numpy fp32 - fp64| {dn:.3g} (ref {ref:.4g})")
        assert dg <= 4 * dn + 1e-6 * abs(ref) + 1e-9, k
    ctx.close()
