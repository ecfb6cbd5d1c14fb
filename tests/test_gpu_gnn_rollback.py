"""A failed GraphNet update leaves the training state unchanged (the fcnet counterpart is
tests/test_gpu_rollback.py).

The fused GNN update snapshots theta / Adam m / v / beta powers before its first step.  The
library's test hook (DDRL_TEST_FAIL_STEP, read at context creation) sets the device error word
before the first step, as a failed launch leaves it: the steps run, the next stats read raises
DdrlError, and theta / m / v / beta powers are bit-identical to their pre-call values.  A healthy
context of the same data then runs the same update normally.
"""
import os

import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import GNN_ENV, GnnOracleRollout, init_gnn_params, make_ctx, run_rollout

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ctx(n, T, **envvars):
    old = {k: os.environ.get(k) for k in envvars}
    os.environ.update({k: str(v) for k, v in envvars.items()})
    try:
        return make_ctx(GNN_ENV, n, T)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _records(n=32, T=10, seed=61):
    ctx, cfg, inst = make_ctx(GNN_ENV, n, T)
    rng = np.random.default_rng(seed)
    params = init_gnn_params(ctx, seed + 1, head_scale=1.0)
    filt = (1000.0, rng.normal(size=cfg.obs_full_dim) * 0.3, np.abs(rng.normal(size=cfg.obs_full_dim)) * 999.0 + 10.0)
    orc, norms, _, _ = run_rollout(ctx, cfg, inst, params, rng, filt, T, orc_cls=GnnOracleRollout)
    rec = orc.flat_records(0, ctx.layout[0])
    ctx.close()
    return rec, norms[0]


def _state(ctx):
    m, v, b1p, b2p = ctx.adam_get(0)
    return [ctx.params_get(0).copy(), np.copy(m), np.copy(v), np.float32(b1p), np.float32(b2p)]


def _run(rec, norm, steps=None, **envvars):
    import torch
    ctx, cfg, _ = _ctx(32, 10, **envvars)
    init_gnn_params(ctx, 62, head_scale=1.0)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norm)
    sh, pe = O.sgd_schedule(np.random.default_rng(7), rec.shape[0], 128, cfg.num_sgd_iter)
    return ctx, cfg, [torch.from_numpy(sh).cuda()], [torch.from_numpy(pe).cuda()]


def test_failed_gnn_update_leaves_state_unchanged():
    from ddrl_amd.native import DdrlError
    rec, norm = _records()
    ctx, cfg, sh, pe = _run(rec, norm, DDRL_TEST_FAIL_STEP=0)
    n = ctx.n_params[0]
    ctx.adam_set(0, np.full(n, 1e-3, np.float32), np.full(n, 1e-3, np.float32), 0.9 ** 3, 0.999 ** 3)
    before = _state(ctx)
    ctx.ppo_update(1, sh, pe, [0.2], max_steps=20)
    with pytest.raises(DdrlError, match="as before the call"):
        ctx.ppo_stats(0, 4)
    for x, y in zip(before, _state(ctx)):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    ctx.close()
    # a healthy context runs the same update normally
    ok, _, sh, pe = _run(rec, norm)
    ok.ppo_update(1, sh, pe, [0.2], max_steps=20)
    assert np.isfinite(ok.ppo_stats(0, 20)).all()
    ok.close()


def test_misplaced_one_launch_step_is_refused_then_three_launches_match_oracle():
    """the one-launch step's placement guard.  DDRL_TEST_GNN_MISPLACE remaps
    the 1-D grid so that the 32 tiles of every (net, backward share) combination are 32
    consecutive blocks, dealt over all eight XCDs.  Every reducer then meets arrival flags of
    this launch carrying another XCC id (gnn.hip gnn_wait_flag) and raises the error word
    instead of summing partials that may sit in another XCD's L2; the per-tile XCC record tells
    the host why.  The call raises, theta / m / v / beta powers are bit-identical to their
    values before it, and the context has switched to the three-launch step: the retried
    update equals a DDRL_GNN_TAIL=0 context bit for bit and meets the fp64 oracle bar of
    tests/test_gpu_gnn.py (strict_params_check)."""
    from ddrl_amd.native import DdrlError
    rec, norm = _records()
    ctx, cfg, sh, pe = _run(rec, norm, DDRL_TEST_GNN_MISPLACE=1)
    n = ctx.n_params[0]
    m0, v0 = np.full(n, 1e-3, np.float32), np.full(n, 1e-3, np.float32)
    ctx.adam_set(0, m0, v0, 0.9 ** 3, 0.999 ** 3)
    before = _state(ctx)
    steps = 12
    ctx.ppo_update(1, sh, pe, [0.2], max_steps=steps)
    with pytest.raises(DdrlError, match="different XCDs.*as before the call.*three-launch"):
        ctx.ppo_stats(0, 4)
    for x, y in zip(before, _state(ctx)):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    ctx.ppo_update(1, sh, pe, [0.2], max_steps=steps)   # retried: three launches
    st = ctx.ppo_stats(0, steps)
    got = _state(ctx)
    ref, _, sh2, pe2 = _run(rec, norm, DDRL_GNN_TAIL=0)
    ref.adam_set(0, m0, v0, 0.9 ** 3, 0.999 ** 3)
    ref.ppo_update(1, sh2, pe2, [0.2], max_steps=steps)
    st_ref = ref.ppo_stats(0, steps)
    for x, y in zip(got, _state(ref)):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    np.testing.assert_array_equal(st, st_ref)
    ref.close()
    # the fp64 oracle bar (tests/test_gpu_gnn.py): same start, same schedule
    from tests.gpu_harness import strict_params_check
    ctx0, _, _ = make_ctx(GNN_ENV, 32, 10)
    params = init_gnn_params(ctx0, 62, head_scale=1.0)
    ctx0.close()
    lay = ctx.layout[0]
    mean, den = norm
    batch = dict(X=rec[:, :92].reshape(-1, 4, 23), node_idx=rec[:, 92].astype(np.int64),
                 actions=rec[:, lay["act"]:lay["act"] + 2], logits=rec[:, lay["logit"]:lay["logit"] + 4],
                 logp=rec[:, lay["logp"]], vf_preds=rec[:, lay["vf"]],
                 adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32), vt=rec[:, lay["vt"]])
    adam = O.Adam(n)
    adam.m, adam.v, adam.b1p, adam.b2p = m0.copy(), v0.copy(), np.float32(0.9 ** 3), np.float32(0.999 ** 3)
    strict_params_check(got[0], "gnn", params, O.gnn_param_shapes(4), batch, sh[0].cpu().numpy(),
                        pe[0].cpu().numpy(), 0.2, steps, adam=adam, msg="gnn after misplacement fallback")
    ctx.close()


@pytest.fixture()
def pg1():
    import socket
    import torch.distributed as dist
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


def test_failed_gnn_ddp_loop_leaves_state_unchanged(pg1):
    """the library's data-parallel loop (ddrl_ppo_update_ddp) on the GraphNet.  Its
    128-row gradient launches reduce in their tail, with bounded waits, so the loop snapshots
    the GNN state too.  With the error word set before step 1's gradient (step 0's Adam has
    already changed theta / m / v / beta powers), the call raises and the state is the
    pre-call state."""
    import torch
    from ddrl_amd.ddp import Comm, NativeDataParallelLearner, native_comm_init
    from ddrl_amd.native import DdrlError
    rec, norm = _records()
    ctx, cfg, _ = _ctx(32, 10, DDRL_TEST_FAIL_STEP=1)
    init_gnn_params(ctx, 62, head_scale=1.0)
    ctx.records_set(0, rec)
    ctx.adv_norm_set(0, *norm)
    before = _state(ctx)
    nat = NativeDataParallelLearner(ctx, Comm("cpu"), 0, 128, "split")
    native_comm_init(ctx, Comm("cpu"))
    shuffle, perms = nat.schedule(np.random.default_rng(1), rec.shape[0], 2)
    with pytest.raises(DdrlError, match="as before the call"):
        nat.learn(torch.from_numpy(shuffle).cuda(), perms, 0.2)
    for x, y in zip(before, _state(ctx)):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    ctx.close()
