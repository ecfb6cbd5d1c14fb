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
