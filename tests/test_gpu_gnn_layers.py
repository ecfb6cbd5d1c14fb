"""f4: the GraphNet's alternate message-passing layers (models/gcn.py: GCN :7-37, MPNN2 :96-150,
GAT1 :153-206, with graph_ops.py:3-26), selected by model_config "gnn_layer" (the reference
selects them by editing models/graph_net.py:20), on the HIP path vs the CPU oracle; MPNN (the
default) is run through the same cases.  The oracle's layers are checked against torch
autograd of the reference's own call() in tests/test_oracle.py.

Tolerances as in test_gpu_gnn.py: rollout outputs 1e-5 relative + 2e-5 absolute, gradients
1e-4 relative to the tensor's largest entry, parameters after 3 Adam steps within 1e-5 for
>= 99.9 % of the entries, and the 100-step schedule within 4x the fp32 oracle's own drift from
the fp64 trajectory (+ 2e-7) and within 1e-5 of the fp32 oracle (gpu_harness.drift_check).
"""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import (GNN_ENV, GnnOracleRollout, init_gnn_params, make_ctx, run_rollout,
                                strict_params_check)

pytestmark = pytest.mark.gpu
LAYERS = ["gcn", "mpnn2", "gat1", "mpnn"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


def _close(a, b, rtol=1e-5, atol=1e-5, msg=""):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=msg)


def _rollout(layer, n, T, seed, head_scale, config=None):
    cfg_ = {"model": {"custom_model": "gnn", "gnn_layer": layer}, **(config or {})}
    ctx, cfg, inst = make_ctx(GNN_ENV, n, T, cfg_)
    rng = np.random.default_rng(seed)
    params = init_gnn_params(ctx, seed + 1, head_scale=head_scale, layer=layer)
    filt = (1000.0, rng.normal(size=cfg.obs_full_dim) * 0.3, np.abs(rng.normal(size=cfg.obs_full_dim)) * 999.0 + 10.0)

    class Orc(GnnOracleRollout):
        pass
    Orc.layer = layer
    orc, norms, a_gpu, a_orc = run_rollout(ctx, cfg, inst, params, rng, filt, T, orc_cls=Orc)
    return ctx, cfg, orc, norms, params, a_gpu, a_orc


def _batch(rec, lay, norms):
    mean, den = norms
    return dict(X=rec[:, :92].reshape(-1, 4, 23), node_idx=rec[:, 92].astype(np.int64),
                actions=rec[:, lay["act"]:lay["act"] + 2], logits=rec[:, lay["logit"]:lay["logit"] + 4],
                logp=rec[:, lay["logp"]], vf_preds=rec[:, lay["vf"]],
                adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32), vt=rec[:, lay["vt"]])


@pytest.mark.parametrize("layer", LAYERS)
def test_layer_rollout_and_forward(layer):
    """Rollout (graph observation, forward, sampling, logp, values) + GAE records of a ragged
    9-env run, and ModelV2.forward through ddrl_policy_forward on 13 random graphs."""
    import torch
    ctx, cfg, orc, norms, params, a_gpu, a_orc = _rollout(layer, 9, 4, 31, head_scale=30.0)
    assert ctx.n_params[0] == sum(int(np.prod(s)) for _, s in O.gnn_param_shapes(4, layer=layer))
    _close(a_gpu, a_orc, msg="env actions")
    lay = ctx.layout[0]
    got, ref = ctx.records_get(0), orc.flat_records(0, lay)
    for name, sl in [("act", slice(lay["act"], lay["act"] + 2)), ("logits", slice(lay["logit"], lay["logit"] + 4)),
                     ("logp", lay["logp"]), ("vf", lay["vf"]), ("adv", lay["adv"]), ("vt", lay["vt"])]:
        _close(got[:, sl], ref[:, sl], rtol=1e-5, atol=2e-5, msg=f"{layer} {name}")
    rng = np.random.default_rng(2)
    n = 13
    X = rng.normal(size=(n, 4, 23)).astype(np.float32)
    node = rng.integers(0, 4, size=n).astype(np.int32)
    logits = torch.zeros((n, 4), device="cuda")
    values = torch.zeros(n, device="cuda")
    ctx.policy_forward(0, torch.from_numpy(X).cuda(), n, logits, values, node_dev=torch.from_numpy(node).cuda())
    ctx.synchronize()
    lr, vr, _ = O.gnn_forward(params, X, node, layer=layer)
    _close(logits.cpu().numpy(), lr, msg=f"{layer} forward logits")
    _close(values.cpu().numpy(), vr, msg=f"{layer} forward value")
    ctx.close()


@pytest.mark.parametrize("layer", LAYERS)
def test_layer_gradient(layer):
    """ddrl_ppo_grad over 128 rows == the oracle gradient of every variable; two ragged row
    sets (50 + 78) sum to it (per-tile partials of ragged tiles)."""
    import torch
    ctx, cfg, orc, norms, params, _, _ = _rollout(layer, 12, 4, 41, head_scale=1.0)
    shapes = O.gnn_param_shapes(4, layer=layer)
    lay = ctx.layout[0]
    rec = orc.flat_records(0, lay)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norms[0])
    rows = np.random.default_rng(3).permutation(rec.shape[0])[:128].astype(np.int32)
    npar = ctx.n_params[0]
    r_all = torch.from_numpy(rows).cuda()
    g_full, g_a, g_b = (torch.zeros(npar, device="cuda") for _ in range(3))
    ctx.ppo_grad(0, r_all, 128, 0.2, g_full)
    ctx.ppo_grad(0, r_all[:50].contiguous(), 50, 0.2, g_a)
    ctx.ppo_grad(0, r_all[50:].contiguous(), 78, 0.2, g_b)
    ctx.synchronize()
    gf = g_full.cpu().numpy()
    np.testing.assert_allclose((g_a + g_b).cpu().numpy(), gf, rtol=1e-4, atol=1e-6 * np.abs(gf).max())
    sl = {k: v[rows] for k, v in _batch(rec, lay, norms[0]).items()}
    logits, value, cache = O.gnn_forward(params, sl["X"], sl["node_idx"], layer=layer)
    dl, dv, _ = O.ppo_loss_rows(logits, value, sl["actions"], sl["logits"], sl["logp"], sl["vf_preds"],
                                sl["adv"], sl["vt"], np.float32(0.2))
    gd = O.gnn_backward(params, cache, dl, dv)
    off = 0
    for name, shape in shapes:
        k = int(np.prod(shape))
        ref = gd[name].reshape(-1)
        assert np.abs(ref).max() > 0, name
        np.testing.assert_allclose(gf[off:off + k], ref, rtol=1e-4, atol=2e-5 * np.abs(ref).max(), err_msg=name)
        off += k
    assert off == npar
    ctx.close()


@pytest.mark.parametrize("layer", LAYERS)
def test_layer_update_3_steps_and_100_step_drift(layer):
    """The fused schedule (grad / reduce / Adam launches): 3 steps against the fp32 oracle
    (parameters, beta powers, learner statistics), then a fresh context runs the whole
    10-epoch schedule of a 1,280-row batch (100 steps) against the fp64 trajectory."""
    import torch
    from tests.gpu_harness import drift_check
    for steps in (3, None):
        ctx, cfg, orc, norms, params, _, _ = _rollout(layer, 32, 10, 51, head_scale=1.0)   # R = 1280, nb = 10
        shapes = O.gnn_param_shapes(4, layer=layer)
        lay = ctx.layout[0]
        rec = orc.flat_records(0, lay)
        ctx.records_set(0, rec)
        ctx.adv_norm_set(0, *norms[0])
        sh, pe = O.sgd_schedule(np.random.default_rng(100), rec.shape[0], 128, cfg.num_sgd_iter)
        batch = _batch(rec, lay, norms[0])
        kw = {"max_steps": steps} if steps else {}
        ctx.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.3], **kw)
        ctx.synchronize()
        if steps:
            adam = O.Adam(ctx.n_params[0], lr=cfg.lr)
            new, stats = O.ppo_update("gnn", params, shapes, adam, batch, sh, pe, np.float32(0.3),
                                      {"entropy_coeff": 0.0, "gnn_layer": layer}, steps=steps)
            got, ref = ctx.params_get(0), O.pack(new, shapes)
            diff = np.abs(got - ref)
            assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref)) >= 0.999 and diff.max() <= 2 * cfg.lr * steps + 1e-5
            strict_params_check(got, "gnn", params, shapes, batch, sh, pe, 0.3, steps, lr=cfg.lr,
                                cfg={"gnn_layer": layer}, msg=layer)
            m, v, b1p, b2p = ctx.adam_get(0)
            assert b1p == np.float32(adam.b1p) and b2p == np.float32(adam.b2p)
            st = ctx.ppo_stats(0, steps)
            for k, s in enumerate(stats):
                want = [s["total_loss"], s["policy_loss"], s["vf_loss"], s["kl"], s["entropy"], s["vf_explained_var"],
                        s["grad_gnorm"]]
                _close(st[k, :7], np.array(want, np.float32), rtol=1e-4, atol=1e-5, msg=f"{layer} stats step {k}")
        else:
            n_steps = cfg.num_sgd_iter * (rec.shape[0] // 128)
            assert n_steps == 100
            drift_check(ctx.params_get(0), "gnn", params, shapes, batch, sh, pe, 0.3, n_steps,
                        cfg={"gnn_layer": layer})
        ctx.close()
