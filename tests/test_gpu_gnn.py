"""GraphNet ("gnn") HIP path vs the CPU oracle (DecentralShared_Graph, one shared leg policy).

Same tolerances as test_gpu_parity.py: rollout outputs 1e-5 relative + 2e-5 absolute;
gradients relative to the tensor's largest entry; parameters after Adam 1e-5 for >= 99.9 %
of the entries.  Ragged tiles (env / row counts not a multiple of 4) are included.
"""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import (GNN_ENV, GnnOracleRollout, init_gnn_params, make_ctx, run_rollout,
                                strict_params_check)

pytestmark = pytest.mark.gpu
SHAPES = O.gnn_param_shapes(4)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


def _close(a, b, rtol=1e-5, atol=1e-5, msg=""):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=msg)


def _filt(D, rng):
    return (1000.0, rng.normal(size=D) * 0.3, np.abs(rng.normal(size=D)) * 999.0 + 10.0)


def _rollout(n, T, seed, head_scale, config=None):
    ctx, cfg, inst = make_ctx(GNN_ENV, n, T, config)
    rng = np.random.default_rng(seed)
    params = init_gnn_params(ctx, seed + 1, head_scale=head_scale)
    orc, norms, a_gpu, a_orc = run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T,
                                           orc_cls=GnnOracleRollout)
    return ctx, cfg, orc, norms, params, a_gpu, a_orc


def _batch(rec, lay, norms):
    mean, den = norms
    return dict(X=rec[:, :92].reshape(-1, 4, 23), node_idx=rec[:, 92].astype(np.int64),
                actions=rec[:, lay["act"]:lay["act"] + 2], logits=rec[:, lay["logit"]:lay["logit"] + 4],
                logp=rec[:, lay["logp"]], vf_preds=rec[:, lay["vf"]],
                adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32), vt=rec[:, lay["vt"]])


def test_gnn_rollout_gae_parity():
    ctx, cfg, orc, norms, params, a_gpu, a_orc = _rollout(9, 4, 31, head_scale=30.0)
    _close(a_gpu, a_orc, msg="env actions")
    lay = ctx.layout[0]
    got = ctx.records_get(0)
    ref = orc.flat_records(0, lay)
    for name, sl in [("X", slice(0, 92)), ("node", 92), ("act", slice(lay["act"], lay["act"] + 2)),
                     ("logits", slice(lay["logit"], lay["logit"] + 4)), ("logp", lay["logp"]),
                     ("vf", lay["vf"]), ("rew", lay["rew"]), ("adv", lay["adv"]), ("vt", lay["vt"])]:
        _close(got[:, sl], ref[:, sl], rtol=1e-5, atol=2e-5, msg=f"gnn {name}")
    _close(ctx.last_values_get(0), orc.last_v[0], msg="bootstrap")
    _close(ctx.adv_norm_get(0), np.array(norms[0], np.float32), rtol=1e-5, atol=1e-6)
    ctx.close()


def test_gnn_policy_forward():
    import torch
    ctx, cfg, inst = make_ctx(GNN_ENV, 4, 2)
    params = init_gnn_params(ctx, 5, head_scale=30.0)
    rng = np.random.default_rng(2)
    n = 13
    X = rng.normal(size=(n, 4, 23)).astype(np.float32)
    node = rng.integers(0, 4, size=n).astype(np.int32)
    logits = torch.zeros((n, 4), device="cuda")
    values = torch.zeros(n, device="cuda")
    ctx.policy_forward(0, torch.from_numpy(X).cuda(), n, logits, values, node_dev=torch.from_numpy(node).cuda())
    ctx.synchronize()
    lr, vr, _ = O.gnn_forward(params, X, node)
    _close(logits.cpu().numpy(), lr)
    _close(values.cpu().numpy(), vr)
    ctx.close()


def test_gnn_grad_and_apply():
    """ppo_grad over 128 rows == oracle gradient; two ragged halves sum to it; ppo_apply ==
    oracle clip + Adam."""
    import torch
    ctx, cfg, orc, norms, params, _, _ = _rollout(12, 4, 41, head_scale=1.0)
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
    b = _batch(rec, lay, norms[0])
    sl = {k: v[rows] for k, v in b.items()}
    logits, value, cache = O.gnn_forward(params, sl["X"], sl["node_idx"])
    dl, dv, _ = O.ppo_loss_rows(logits, value, sl["actions"], sl["logits"], sl["logp"], sl["vf_preds"],
                                sl["adv"], sl["vt"], np.float32(0.2))
    gd = O.gnn_backward(params, cache, dl, dv)
    off = 0
    for name, shape in SHAPES:
        k = int(np.prod(shape))
        ref = gd[name].reshape(-1)
        np.testing.assert_allclose(gf[off:off + k], ref, rtol=1e-4, atol=2e-5 * max(np.abs(ref).max(), 1e-12),
                                   err_msg=name)
        off += k
    assert off == npar
    gref = O.pack(gd, SHAPES)
    ctx.ppo_apply(0, g_full)
    ctx.synchronize()
    adam = O.Adam(npar)
    clipped, _ = O.clip_by_global_norm([gref], 0.5)
    ref = adam.apply(O.pack(params, SHAPES), clipped[0])
    got = ctx.params_get(0)
    diff = np.abs(got - ref)
    assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref)) >= 0.999 and diff.max() <= 2 * 3e-4 + 1e-5
    rest = np.setdiff1d(np.arange(rec.shape[0], dtype=np.int32), rows)
    sh1 = np.concatenate([rows, rest]).astype(np.int32)
    strict_params_check(got, "gnn", params, SHAPES, b, sh1, np.arange(sh1.size // 128, dtype=np.int32)[None],
                        0.2, 1, msg="gnn apply")
    ctx.close()


def test_gnn_update_parity():
    """Fused GNN schedule (grad / reduce / Adam launches) for 3 minibatch steps."""
    import torch
    ctx, cfg, orc, norms, params, _, _ = _rollout(16, 10, 51, head_scale=1.0)   # R = 640, nb = 5
    lay = ctx.layout[0]
    rec = orc.flat_records(0, lay)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norms[0])
    sh, pe = O.sgd_schedule(np.random.default_rng(100), rec.shape[0], 128, cfg.num_sgd_iter)
    steps = 3
    ctx.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.3], max_steps=steps)
    ctx.synchronize()
    adam = O.Adam(ctx.n_params[0], lr=cfg.lr)
    new, stats = O.ppo_update("gnn", params, SHAPES, adam, _batch(rec, lay, norms[0]), sh, pe, np.float32(0.3),
                              {"entropy_coeff": 0.0}, steps=steps)
    got = ctx.params_get(0)
    ref = O.pack(new, SHAPES)
    diff = np.abs(got - ref)
    frac = np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref))
    assert frac >= 0.999 and diff.max() <= 2 * cfg.lr * steps + 1e-5, (frac, diff.max())
    strict_params_check(got, "gnn", params, SHAPES, _batch(rec, lay, norms[0]), sh, pe, 0.3, steps, lr=cfg.lr,
                        msg="gnn update")
    m, v, b1p, b2p = ctx.adam_get(0)
    assert b1p == np.float32(adam.b1p) and b2p == np.float32(adam.b2p)
    st = ctx.ppo_stats(0, steps)
    for k, s in enumerate(stats):
        ref = [s["total_loss"], s["policy_loss"], s["vf_loss"], s["kl"], s["entropy"], s["vf_explained_var"],
               s["grad_gnorm"]]
        _close(st[k, :7], np.array(ref, np.float32), rtol=1e-4, atol=1e-5, msg=f"stats step {k}")
    ctx.close()


def test_gnn_update_long_horizon():
    """The whole 10-epoch schedule of a 1,280-row batch (100 sequential grad / reduce / Adam
    steps) against the fp64 trajectory (tests/gpu_harness.drift_check: HIP deviation <= 4x
    the numpy fp32 deviation + 2e-7, and within 1e-5 of the fp32 oracle); learner statistics
    of every step within 1e-4 relative of the fp64 ones."""
    import torch
    from tests.gpu_harness import drift_check
    ctx, cfg, orc, norms, params, _, _ = _rollout(32, 10, 61, head_scale=1.0)   # R = 1280, nb = 10
    lay = ctx.layout[0]
    rec = orc.flat_records(0, lay)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norms[0])
    sh, pe = O.sgd_schedule(np.random.default_rng(7), rec.shape[0], 128, cfg.num_sgd_iter)
    steps = cfg.num_sgd_iter * (rec.shape[0] // 128)
    assert steps == 100
    ctx.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.2])
    ctx.synchronize()
    _, _, _, st64, _ = drift_check(ctx.params_get(0), "gnn", params, SHAPES, _batch(rec, lay, norms[0]), sh, pe,
                                   0.2, steps)
    st = ctx.ppo_stats(0, steps).astype(np.float64)
    for col, k in [(1, "policy_loss"), (2, "vf_loss"), (3, "kl"), (4, "entropy"), (6, "grad_gnorm")]:
        ref = np.array([s[k] for s in st64])
        assert np.all(np.abs(st[:, col] - ref) <= 1e-4 * np.abs(ref) + 1e-6), k
    ctx.close()


def test_gnn_update_across_record_chunks():
    """The fused GNN update gathers the records of each run of 1024 minibatch steps into one
    chunk (k_gnn_gather, GNN_CHUNK_STEPS).  A 1,030-step schedule (103 epochs of a 1,280-row
    batch) at lr = 0 keeps the weights fixed, so every step's learner statistics are the loss
    of its own minibatch at the initial weights: steps on both sides of the chunk boundary
    are compared with the oracle one by one (no trajectory drift), and the weights must come
    back unchanged bit for bit."""
    import torch
    ctx, cfg, orc, norms, params, _, _ = _rollout(32, 10, 71, head_scale=1.0,
                                                  config={"num_sgd_iter": 103, "lr": 0.0})
    lay = ctx.layout[0]
    rec = orc.flat_records(0, lay)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norms[0])
    sh, pe = O.sgd_schedule(np.random.default_rng(9), rec.shape[0], 128, cfg.num_sgd_iter)
    nb = rec.shape[0] // 128
    steps = cfg.num_sgd_iter * nb
    assert steps == 1030
    p0 = ctx.params_get(0).copy()
    ctx.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.2])
    ctx.synchronize()
    np.testing.assert_array_equal(ctx.params_get(0), p0)
    st = ctx.ppo_stats(0, steps)
    batch = _batch(rec, lay, norms[0])
    for k in [0, 1, 1022, 1023, 1024, 1025, 1029]:
        e, b = divmod(k, nb)
        _, stats = O.ppo_update("gnn", params, SHAPES, O.Adam(ctx.n_params[0], lr=0.0), batch, sh,
                                pe[e:e + 1, b:b + 1], np.float32(0.2), {"entropy_coeff": 0.0}, steps=1)
        s0 = stats[0]
        ref = [s0["total_loss"], s0["policy_loss"], s0["vf_loss"], s0["kl"], s0["entropy"], s0["vf_explained_var"],
               s0["grad_gnorm"]]
        _close(st[k, :7], np.array(ref, np.float32), rtol=1e-4, atol=1e-5, msg=f"stats step {k}")
    ctx.close()


def test_gnn_one_launch_step_matches_three_launch_step(monkeypatch):
    """Round 4: the GNN training step in ONE launch (gnn.hip gnn_tail: the 32 tiles of each
    (net, backward share) combination on one XCD reduce their partials through its L2, then a
    tagged norm^2 granule per reducer crosses XCDs, then clip + Adam) against the three-launch
    step (DDRL_GNN_TAIL=0: k_gnn -> k_gnn_reduce -> k_gnn_adam).  The gradient of a minibatch
    (ddrl_ppo_grad of 128 rows: the reduction in the tail, Adam left to the caller) is bit-identical
    -- every parameter's 32 partials are summed in the same tile order.  The global norm sums
    the same squares in another grouping, so the 100-step schedule agrees to fp32 rounding of the
    clip scale: parameters within 2e-6, learner statistics within 1e-5 relative + 2e-6; both paths are
    held to the fp64 oracle by the other tests of this file."""
    import torch
    from ddrl_amd import native as N
    ctx0, cfg, orc, norms, params, _, _ = _rollout(32, 10, 81, head_scale=1.0)
    ctx0.close()
    ctxs = []
    for tail in ("1", "0"):
        monkeypatch.setenv("DDRL_GNN_TAIL", tail)
        c = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
        lay = c.layout[0]
        rec = orc.flat_records(0, lay)
        c.records_set(0, rec)
        c.adv_norm_set(0, *norms[0])
        c.params_set(0, O.pack(params, SHAPES))
        ctxs.append(c)
    monkeypatch.delenv("DDRL_GNN_TAIL")
    sh, pe = O.sgd_schedule(np.random.default_rng(17), rec.shape[0], 128, cfg.num_sgd_iter)
    steps = cfg.num_sgd_iter * (rec.shape[0] // 128)
    rows = torch.from_numpy(sh[:128].copy()).cuda()
    grads = []
    for c in ctxs:
        g = torch.zeros(c.n_params[0], device="cuda")
        c.ppo_grad(0, rows, 128, 0.2, g)
        c.synchronize()
        grads.append(g.cpu().numpy())
        c.ppo_update(1, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()], [0.2])
        c.synchronize()
    np.testing.assert_array_equal(grads[0], grads[1])
    assert np.abs(grads[0]).max() > 0
    a, b = ctxs
    pa, pb = a.params_get(0), b.params_get(0)
    assert not np.array_equal(pa, O.pack(params, SHAPES))
    np.testing.assert_allclose(pa, pb, rtol=0, atol=2e-6)
    ma, va, b1a, b2a = a.adam_get(0)
    mb, vb, b1b, b2b = b.adam_get(0)
    assert (b1a, b2a) == (b1b, b2b)
    np.testing.assert_allclose(a.ppo_stats(0, steps), b.ppo_stats(0, steps), rtol=1e-5, atol=2e-6)
    for c in ctxs:
        c.close()
