"""The "cup" model (models/coupling_net_glorot_uniform_init.py:11-137) on the HIP path vs the
CPU oracle, through the C-ABI (needs an MI355X).

The cup model is the fcnet of the SharedDecentralLegID env's 19 features whose action means
are scaled by a trainable [4][A] leg-coupling table, row = the agent's leg index.  Covered:
rollout + GAE records (coupled logits, the leg index field), the fused update (both row-split
halves carry the coupling gradient), the data-parallel gradient of one minibatch (the
coupling table's gradient included) and ModelV2.forward through the "cup" ModelCatalog class.
Tolerances as in test_gpu_parity.py.
"""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import (CUP_CONFIG, CUP_ENV, CupOracleRollout, init_cup_params, make_ctx, run_rollout,
                                strict_params_check)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


def _filt(D, rng):
    return (1000.0, rng.normal(size=D) * 0.3, np.abs(rng.normal(size=D)) * 999.0 + 10.0)


def _batch(rec, lay, d, A, adv_norm):
    mean, den = adv_norm
    return dict(obs=rec[:, lay["obs"]:lay["obs"] + d], actions=rec[:, lay["act"]:lay["act"] + A],
                logits=rec[:, lay["logit"]:lay["logit"] + 2 * A], logp=rec[:, lay["logp"]],
                vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                vt=rec[:, lay["vt"]], leg=rec[:, lay["leg"]].astype(np.int64))


def _rollout(n, T, seed, head_scale=30.0):
    ctx, cfg, inst = make_ctx(CUP_ENV, n, T, CUP_CONFIG)
    assert cfg.leg_coupling == 1 and cfg.obs_dim[0] == 19
    rng = np.random.default_rng(seed)
    params = init_cup_params(ctx, cfg, seed + 1, head_scale=head_scale)
    orc, norms, a_gpu, a_orc = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T,
                                           orc_cls=CupOracleRollout)
    return ctx, cfg, params, orc, norms, a_gpu, a_orc


def test_cup_layout_and_param_count():
    ctx, cfg, inst = make_ctx(CUP_ENV, 8, 2, CUP_CONFIG)
    shapes = O.cup_param_shapes(19, 2)
    assert ctx.n_params[0] == sum(int(np.prod(s)) for _, s in shapes) == 11205 + 8
    lay = ctx.layout[0]
    assert lay["leg"] == lay["rew"] + 1 and lay["stride"] % 4 == 0 and lay["leg"] < lay["stride"]
    ctx.close()
    # the plain LegID env keeps its one-hot fcnet input and has no leg field
    ctx, cfg, _ = make_ctx(CUP_ENV, 8, 2)
    assert cfg.leg_coupling == 0 and cfg.obs_dim[0] == 23 and ctx.layout[0]["leg"] == -1
    ctx.close()


def test_cup_rollout_gae_parity():
    # head scale 20: the coupling (up to 1.5x) brings the means to the 30x-head scale of the
    # other rollout tests; logp = -z^2/2 - log sd with z = (a - mu) / sd loses
    # ulp(mu) / sd to cancellation, so larger means would only test fp32 conditioning
    n, T = 24, 4
    ctx, cfg, params, orc, norms, a_gpu, a_orc = _rollout(n, T, 31, head_scale=20.0)
    np.testing.assert_allclose(a_gpu, a_orc, rtol=1e-5, atol=1e-5, err_msg="env actions")
    lay = ctx.layout[0]
    got = ctx.records_get(0)
    ref = orc.flat_records(0, lay)
    A = 2
    for name, sl in [("obs", slice(0, 19)), ("act", slice(lay["act"], lay["act"] + A)),
                     ("logits", slice(lay["logit"], lay["logit"] + 2 * A)), ("logp", lay["logp"]),
                     ("vf", lay["vf"]), ("rew", lay["rew"]), ("adv", lay["adv"]), ("vt", lay["vt"])]:
        np.testing.assert_allclose(got[:, sl], ref[:, sl], rtol=1e-5, atol=2e-5, err_msg=name)
    np.testing.assert_array_equal(got[:, lay["leg"]], ref[:, lay["leg"]])
    # the coupling acts: legs with negative coupling flip the sign of the mean
    raw, _, _ = O.ffn_forward(params[0], ref[:, :19])
    np.testing.assert_allclose(ref[:, lay["logit"]:lay["logit"] + A],
                               raw[:, :A] * params[0]["leg_coupling"][ref[:, lay["leg"]].astype(int)],
                               rtol=1e-6, atol=1e-7)
    ctx.close()


@pytest.mark.parametrize("steps", [1, 3])
def test_cup_fused_update_parity(steps):
    import torch
    n, T = 32, 4
    ctx, cfg, params, orc, norms, _, _ = _rollout(n, T, 41, head_scale=1.0)
    lay = ctx.layout[0]
    ref = orc.flat_records(0, lay)
    ctx.records_set(0, ref)
    ctx.adv_norm_set(0, *norms[0])
    sh, pe = O.sgd_schedule(np.random.default_rng(5), T * lay["C"], 128, cfg.num_sgd_iter)
    ctx.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.25], max_steps=steps)
    ctx.synchronize()
    shapes = O.cup_param_shapes(19, 2)
    adam = O.Adam(sum(int(np.prod(s)) for _, s in shapes), lr=cfg.lr)
    new, stats = O.ppo_update("cup", params[0], shapes, adam, _batch(ref, lay, 19, 2, norms[0]), sh, pe,
                              np.float32(0.25), {"entropy_coeff": 0.0}, steps=steps)
    got = ctx.params_get(0)
    want = O.pack(new, shapes)
    diff = np.abs(got - want)
    assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(want)) >= 0.999, diff.max()
    assert diff.max() <= 2 * cfg.lr * steps + 1e-5
    strict_params_check(got, "cup", params[0], shapes, _batch(ref, lay, 19, 2, norms[0]), sh, pe, 0.25, steps,
                        lr=cfg.lr, msg="cup")
    # the coupling table itself moved, and matches
    np.testing.assert_allclose(got[-8:], want[-8:], rtol=1e-5, atol=1e-5)
    assert np.abs(got[-8:] - O.pack(params[0], shapes)[-8:]).max() > 0
    m, v, b1p, b2p = ctx.adam_get(0)
    assert np.all(v[-8:] > 0), "coupling entries carry Adam state"
    st = ctx.ppo_stats(0, steps)
    for k, s in enumerate(stats):
        r = [s["total_loss"], s["policy_loss"], s["vf_loss"], s["kl"], s["entropy"],
             s["vf_explained_var"], s["grad_gnorm"]]
        np.testing.assert_allclose(st[k, :7], np.array(r, np.float32), rtol=1e-4, atol=1e-5)
    ctx.close()


def test_cup_ddp_grad_matches_oracle():
    import torch
    n, T = 32, 4
    ctx, cfg, params, orc, norms, _, _ = _rollout(n, T, 51, head_scale=1.0)
    lay = ctx.layout[0]
    ref = orc.flat_records(0, lay)
    ctx.records_set(0, ref)
    ctx.adv_norm_set(0, *norms[0])
    rows = np.random.default_rng(3).permutation(T * lay["C"])[:128].astype(np.int32)
    g = torch.zeros(ctx.n_params[0], device="cuda")
    ctx.ppo_grad(0, torch.from_numpy(rows).cuda(), 128, 0.2, g)
    ctx.synchronize()
    b = {k: v[rows] for k, v in _batch(ref, lay, 19, 2, norms[0]).items()}
    logits, value, cache = O.cup_forward(params[0], b["obs"], b["leg"])
    dl, dv, _ = O.ppo_loss_rows(logits, value, b["actions"], b["logits"], b["logp"], b["vf_preds"],
                                b["adv"], b["vt"], np.float32(0.2))
    gref = O.pack(O.cup_backward(params[0], cache, dl, dv), O.cup_param_shapes(19, 2))
    gg = g.cpu().numpy()
    np.testing.assert_allclose(gg, gref, rtol=1e-4, atol=2e-5 * np.abs(gref).max())
    np.testing.assert_allclose(gg[-8:], gref[-8:], rtol=1e-4, atol=1e-6)
    ctx.close()


def test_cup_model_forward():
    import torch
    from ddrl_amd.models import ModelCatalog
    ctx, cfg, inst = make_ctx(CUP_ENV, 8, 2, CUP_CONFIG)
    params = init_cup_params(ctx, cfg, 61)
    cls = ModelCatalog.get("cup")
    m = cls(None, None, 4, {"fcnet_hiddens": [64, 64], "fcnet_activation": "tanh"}, "policy_legs", ctx=ctx, pid=0)
    rng = np.random.default_rng(0)
    x = rng.normal(size=(203, 19)).astype(np.float32)
    leg = rng.integers(0, 4, size=(203, 1))
    logits, _ = m.forward({"obs": (leg, x)}, [], None)
    values = m.value_function()
    torch.cuda.synchronize()
    lr, vr, _ = O.cup_forward(params[0], x, leg)
    np.testing.assert_allclose(logits.cpu().numpy(), lr, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(values.cpu().numpy(), vr, rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError):
        m.forward({"obs": (leg + 4, x)}, [], None)
    ctx.close()


def test_cup_update_long_horizon():
    """"cup" model over its whole 10-epoch schedule of a 1,280-row batch (100 fused steps)
    against the fp64 trajectory (tests/gpu_harness.drift_check), coupling table included."""
    import torch
    from tests.gpu_harness import drift_check
    n, T = 32, 10
    ctx, cfg, params, orc, norms, _, _ = _rollout(n, T, 43, head_scale=1.0)
    lay = ctx.layout[0]
    ref = orc.flat_records(0, lay)
    ctx.records_set(0, ref)
    ctx.adv_norm_set(0, *norms[0])
    sh, pe = O.sgd_schedule(np.random.default_rng(9), T * lay["C"], 128, cfg.num_sgd_iter)
    steps = cfg.num_sgd_iter * (T * lay["C"] // 128)
    assert steps == 100
    ctx.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.25])
    ctx.synchronize()
    shapes = O.cup_param_shapes(19, 2)
    drift_check(ctx.params_get(0), "cup", params[0], shapes, _batch(ref, lay, 19, 2, norms[0]), sh, pe, 0.25, steps)
    ctx.close()
