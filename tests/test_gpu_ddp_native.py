"""The library-side data-parallel loop (ddrl_comm_init + ddrl_ppo_update_ddp: per minibatch
gradient -> ncclAllReduce -> clip + Adam, enqueued from C++) against the Python
DataParallelLearner driving ddrl_ppo_grad / ddrl_ppo_apply, on a one-rank RCCL communicator.

Both run the same kernels on the same records in the same order, and a one-rank all-reduce
is a copy, so parameters, Adam state (through a second update) and learner statistics must
agree bit for bit.  grad_scale != 1 (the "local" mode's 1 / ranks) is covered by forcing it
on both learners: the Python side multiplies with torch, the library inside the Adam kernel.
"""
import os
import socket

import numpy as np
import pytest

from tests.gpu_harness import (GnnOracleRollout, init_gnn_params, init_params, make_ctx,
                               run_rollout)
from oracle import ddrl_oracle as O

pytestmark = pytest.mark.gpu

GNN_ENV = "QuantrupedMultiEnv_DecentralShared_Graph"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture()
def pg1():
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


def _filt(D, rng):
    return (1000.0, rng.normal(size=D) * 0.3, np.abs(rng.normal(size=D)) * 999.0 + 10.0)


def _pair(env, n, T, gnn):
    """Context a after a rollout, context b with a's records, advantage norm and weights."""
    ctx, cfg, inst = make_ctx(env, n, T)
    rng = np.random.default_rng(41)
    if gnn:
        params = init_gnn_params(ctx, 42, head_scale=1.0)
        run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T, orc_cls=GnnOracleRollout)
    else:
        params = init_params(ctx, cfg, 42, head_scale=1.0)
        run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    ctx_b, _, _ = make_ctx(env, n, T)
    ctx_b.params_set(0, ctx.params_get(0))
    ctx_b.records_set(0, ctx.records_get(0))
    ctx_b.adv_norm_set(0, *ctx.adv_norm_get(0))
    return ctx, ctx_b


@pytest.mark.parametrize("env,n,T,gnn,mode,gscale", [
    ("QuantrupedMultiEnv_SharedDecentral", 32, 4, False, "split", 1.0),
    ("QuantrupedMultiEnv_SharedDecentral", 32, 4, False, "local", 0.5),
    (GNN_ENV, 16, 4, True, "split", 1.0),
    (GNN_ENV, 16, 4, True, "local", 0.25),
])
def test_native_ddp_loop_matches_python_learner(pg1, env, n, T, gnn, mode, gscale):
    import torch
    from ddrl_amd.ddp import (Comm, DataParallelLearner, HipBackend, NativeDataParallelLearner,
                              native_comm_init)
    ctx_a, ctx_b = _pair(env, n, T, gnn)
    comm = Comm("cpu")
    py = DataParallelLearner(HipBackend(ctx_a), comm, 0, 128, mode)
    nat = NativeDataParallelLearner(ctx_b, comm, 0, 128, mode)
    py.grad_scale = nat.grad_scale = gscale
    native_comm_init(ctx_b, comm)
    R = ctx_a.records_get(0).shape[0]
    grad = torch.zeros(ctx_a.n_params[0], device="cuda")
    for it in range(2):   # the second update starts from non-zero Adam moments
        sh, pe = O.sgd_schedule(np.random.default_rng(7 + it), R, 128, 2)
        sh_dev = torch.from_numpy(sh).cuda()
        kl_a = py.learn(sh_dev, pe, 0.2, grad)
        kl_b = nat.learn(sh_dev, pe, 0.2)
        ctx_a.synchronize()
        ctx_b.synchronize()
        np.testing.assert_array_equal(ctx_b.params_get(0), ctx_a.params_get(0))
        np.testing.assert_array_equal(ctx_b.ppo_stats(0, pe.shape[1]), ctx_a.ppo_stats(0, pe.shape[1]))
        assert kl_a == kl_b
    # the library's all-reduce entry on its own: one rank sums to itself
    x = torch.arange(1000, dtype=torch.float32, device="cuda")
    ctx_b.comm_allreduce(x)
    ctx_b.synchronize()
    np.testing.assert_array_equal(x.cpu().numpy(), np.arange(1000, dtype=np.float32))
    ctx_a.close()
    ctx_b.close()


def test_native_ddp_argument_errors(pg1):
    import torch
    from ddrl_amd.native import DdrlError
    ctx, _, _ = make_ctx("QuantrupedMultiEnv_SharedDecentral", 8, 2)
    sh = torch.zeros(64, dtype=torch.int32, device="cuda")
    with pytest.raises(DdrlError, match="communicator"):
        ctx.ppo_update_ddp(0, sh, np.zeros((1, 1), np.int32), 64, 0.2, 1.0)
    from ddrl_amd.ddp import Comm, native_comm_init
    native_comm_init(ctx, Comm("cpu"))
    with pytest.raises(DdrlError, match="already"):
        native_comm_init(ctx, Comm("cpu"))
    with pytest.raises(DdrlError, match="slot"):
        ctx.ppo_update_ddp(0, sh, np.full((1, 1), 5, np.int32), 64, 0.2, 1.0)
    with pytest.raises(DdrlError, match="rows_per_rank"):
        ctx.ppo_update_ddp(0, sh, np.zeros((1, 1), np.int32), 200, 0.2, 1.0)
    ctx.close()


def test_grad_launches_across_epoch_wrap():
    """Exchange granules carry a 12-bit per-context launch epoch and are cleared only when it
    wraps (every 4,095 update launches).  Alternate two minibatches over 4,100 gradient
    launches (row split: the partial-gradient exchange is live) and check the launches
    around the wrap against the first two: a stale granule taken for a fresh one would
    mix the other minibatch's partial sums in."""
    import torch
    ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_SharedDecentral", 32, 4)
    rng = np.random.default_rng(3)
    params = init_params(ctx, cfg, 5, head_scale=1.0)
    run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), 4)
    R = ctx.records_get(0).shape[0]
    perm = torch.from_numpy(np.random.default_rng(9).permutation(R).astype(np.int32)).cuda()
    rows = [perm[:128], perm[128:256]]
    g = torch.zeros(ctx.n_params[0], device="cuda")
    ref = []
    for i in range(4100):
        ctx.ppo_grad(0, rows[i & 1], 128, 0.2, g, -1)
        if i < 2:
            ctx.synchronize()
            ref.append(g.clone())
        elif 4093 <= i or i % 1024 == 0:
            ctx.synchronize()
            assert torch.equal(g, ref[i & 1]), f"gradient launch {i}"
    assert not torch.equal(ref[0], ref[1])
    ctx.close()
