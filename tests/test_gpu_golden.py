"""The HIP path against the committed oracle vectors (tests/golden/oracle_golden.npz), through
the C-ABI (needs an MI355X).  Fixed targets, independent of the live oracle:

  * fcnet forward (ModelV2.forward / value_function) of the Local policy;
  * GAE + StandardizeFields of a replayed fragment (records, dones and V(s_T) set directly);
  * one fused PPO minibatch step (ddrl_ppo_update) and the data-parallel gradient
    (ddrl_ppo_grad) for the fcnet, "cup" and GraphNet models: parameters after clip + Adam,
    the gradient, and the learner statistics.

The minibatch is placed at record rows 0..127 with shuffle = identity and one minibatch per
epoch, and the advantage normalization is set to (0, 1), so the kernel sees exactly the
fixture's batch.  Tolerances as tests/test_gpu_parity.py: outputs 1e-5 relative + 2e-5
absolute; gradients 1e-4 relative to the tensor's largest entry; parameters after Adam
within 1e-5 for >= 99.9 % of the entries and within 2 lr everywhere; statistics 1e-4.
"""
import os

import numpy as np
import pytest

from tests.gpu_harness import CUP_CONFIG, CUP_ENV, GNN_ENV, make_ctx

pytestmark = pytest.mark.gpu
Z = os.path.join(os.path.dirname(__file__), "golden", "oracle_golden.npz")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from ddrl_amd import build
    build.build()


@pytest.fixture(scope="module")
def z():
    return np.load(Z)


def _records(ctx, p, rows, fields):
    lay = ctx.layout[p]
    rec = np.zeros((lay["C"] * ctx.cfg.frag_len, lay["stride"]), np.float32)
    assert rec.shape[0] >= rows
    for name, val in fields.items():
        val = np.asarray(val, np.float32)
        off = lay[name]
        if val.ndim == 1:
            rec[:len(val), off] = val
        else:
            rec[:len(val), off:off + val.shape[1]] = val
    return rec


def _step_and_grad(ctx, pre, z, kl, shapes_n):
    """Fused step (max_steps = 1) on rows 0..127, then the data-parallel gradient of the same
    rows from the original parameters; returns (new params, stats, grad)."""
    import torch
    R = ctx.layout[0]["C"] * ctx.cfg.frag_len
    assert R == 128, R
    ident = torch.arange(128, dtype=torch.int32, device="cuda")
    perm = torch.zeros((ctx.cfg.num_sgd_iter, 1), dtype=torch.int32, device="cuda")
    ctx.adv_norm_set(0, 0.0, 1.0)
    p0 = ctx.params_get(0)
    P = ctx.cfg.n_policies
    ctx.ppo_update(1, [ident] + [None] * (P - 1), [perm] + [None] * (P - 1), [kl] * P, max_steps=1)
    ctx.synchronize()
    new = ctx.params_get(0)
    st = ctx.ppo_stats(0, 1)[0]
    ctx.params_set(0, p0)
    g = torch.zeros(shapes_n, device="cuda")
    ctx.ppo_grad(0, ident, 128, kl, g)
    ctx.synchronize()
    return new, st, g.cpu().numpy()


def _check_step(new, st, g, z, pre, lr=3e-4):
    want = z[pre + "new_params"]
    diff = np.abs(new - want)
    assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(want)) >= 0.999, diff.max()
    assert diff.max() <= 2 * lr + 1e-5
    gref = z[pre + "grad"]
    np.testing.assert_allclose(g, gref, rtol=1e-4, atol=1e-4 * np.abs(gref).max())
    np.testing.assert_allclose(st[:7], z[pre + "stats"], rtol=1e-4, atol=1e-5)


def test_golden_ffn_forward(z):
    import torch
    ctx, cfg, _ = make_ctx("QuantrupedMultiEnv_Local", 8, 2)
    ctx.params_set(1, z["ffn_params"])
    x = torch.from_numpy(z["ffn_obs"]).cuda()
    logits = torch.zeros((64, 4), device="cuda")
    values = torch.zeros(64, device="cuda")
    ctx.policy_forward(1, x, 64, logits, values)
    ctx.synchronize()
    np.testing.assert_allclose(logits.cpu().numpy(), z["ffn_logits"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(values.cpu().numpy(), z["ffn_value"], rtol=1e-5, atol=2e-5)
    ctx.close()


def test_golden_gae(z):
    T, C = z["gae_rew"].shape
    ctx, cfg, _ = make_ctx("QuantrupedMultiEnv_Centralized", C, T)   # one policy, k = 1: C = N
    lay = ctx.layout[0]
    rec = np.zeros((T * C, lay["stride"]), np.float32)
    rec[:, lay["rew"]] = z["gae_rew"].reshape(-1)
    rec[:, lay["vf"]] = z["gae_vf"].reshape(-1)
    ctx.records_set(0, rec)
    ctx.done_set(z["gae_dones"].astype(np.uint8))
    ctx.last_values_set(0, z["gae_last_v"])
    ctx.gae()
    got = ctx.records_get(0)
    np.testing.assert_allclose(got[:, lay["adv"]].reshape(T, C), z["gae_adv"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(got[:, lay["vt"]].reshape(T, C), z["gae_vt"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(ctx.adv_norm_get(0), z["gae_norm"], rtol=1e-5, atol=1e-6)
    ctx.close()


def test_golden_ffn_step(z):
    # Local, 32 envs x T = 4: R = 128 rows for policy 0
    ctx, cfg, _ = make_ctx("QuantrupedMultiEnv_Local", 32, 4)
    pre = "ffn_step_"
    ctx.params_set(0, z[pre + "params"])
    ctx.records_set(0, _records(ctx, 0, 128, {"obs": z[pre + "obs"], "act": z[pre + "actions"],
                                               "logit": z[pre + "logits"], "logp": z[pre + "logp"],
                                               "vf": z[pre + "vf_preds"], "adv": z[pre + "adv"],
                                               "vt": z[pre + "vt"]}))
    new, st, g = _step_and_grad(ctx, pre, z, 0.3, ctx.n_params[0])
    _check_step(new, st, g, z, pre)
    ctx.close()


def test_golden_cup_step(z):
    # SharedDecentralLegID + "cup", 32 envs x 4 legs x T = 1: R = 128 rows
    ctx, cfg, _ = make_ctx(CUP_ENV, 32, 1, CUP_CONFIG)
    pre = "cup_"
    ctx.params_set(0, z[pre + "params"])
    ctx.records_set(0, _records(ctx, 0, 128, {"obs": z[pre + "obs"], "act": z[pre + "actions"],
                                               "logit": z[pre + "logits"], "logp": z[pre + "logp"],
                                               "vf": z[pre + "vf_preds"], "adv": z[pre + "adv"],
                                               "vt": z[pre + "vt"], "leg": z[pre + "leg"]}))
    new, st, g = _step_and_grad(ctx, pre, z, 0.2, ctx.n_params[0])
    _check_step(new, st, g, z, pre)
    ctx.close()


def test_golden_gnn_forward_and_step(z):
    import torch
    # DecentralShared_Graph, 32 envs x 4 nodes x T = 1: R = 128 rows
    ctx, cfg, _ = make_ctx(GNN_ENV, 32, 1)
    pre = "gnn_"
    ctx.params_set(0, z[pre + "params"])
    X = z[pre + "X"].reshape(128, 92)
    node = z[pre + "node_idx"]
    logits = torch.zeros((128, 4), device="cuda")
    values = torch.zeros(128, device="cuda")
    ctx.policy_forward(0, torch.from_numpy(z[pre + "X"]).cuda(), 128, logits, values,
                       node_dev=torch.from_numpy(node.astype(np.int32)).cuda())
    ctx.synchronize()
    np.testing.assert_allclose(logits.cpu().numpy(), z["gnn_fwd_logits"], rtol=1e-5, atol=2e-5)
    np.testing.assert_allclose(values.cpu().numpy(), z["gnn_fwd_value"], rtol=1e-5, atol=2e-5)
    obs = np.concatenate([X, node[:, None].astype(np.float32)], 1)   # record obs field: X ++ node
    ctx.records_set(0, _records(ctx, 0, 128, {"obs": obs, "act": z[pre + "actions"], "logit": z[pre + "logits"],
                                               "logp": z[pre + "logp"], "vf": z[pre + "vf_preds"],
                                               "adv": z[pre + "adv"], "vt": z[pre + "vt"]}))
    new, st, g = _step_and_grad(ctx, pre, z, 0.2, ctx.n_params[0])
    _check_step(new, st, g, z, pre)
    ctx.close()
