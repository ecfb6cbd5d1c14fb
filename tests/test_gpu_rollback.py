"""a failed fcnet update leaves the training state unchanged, and the
exchange protocol follows the placement the hardware actually gives.

  * The library's test hook (DDRL_TEST_FAIL_STEP, read at context creation) starts a fused
    launch with the error word set, as an exchange abandoned at its 3 s bound leaves it: every
    workgroup runs its steps, none writes its weights back (the word is checked before the
    write-back), and the host restores the snapshot it took before the launch.  (The hook is
    host-side: a per-step compare inside the kernel measured 0.18 us per step.)
    The call raises DdrlError and theta / Adam m / v / beta powers of every policy are
    bit-identical to their values before the call; the next update on a healthy context
    runs normally.
  * The library-side data-parallel loop (ddrl_ppo_update_ddp, one-rank RCCL communicator)
    with the error word set before step k's gradient launch: that Adam launch and every later
    one see the word and skip, the call raises, and the state is the pre-call state.
  * The formally defined exchange (relaxed agent-scope atomics, ppo_ffn_atomic.hip) that the
    context switches to when the recorded XCC ids (HW_REG_XCC_ID, one per block) show a
    policy's workgroups on different XCDs: forced with DDRL_XCHG=atomic, it gives results
    bit-identical to the default protocol's (both exchange the same fp32 values).
"""
import os
import socket

import numpy as np
import pytest

from tests.gpu_harness import init_params, make_ctx, run_rollout

pytestmark = pytest.mark.gpu
ENV = "QuantrupedMultiEnv_Local"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _filt(D, rng):
    return (1000.0, rng.normal(size=D) * 0.3, np.abs(rng.normal(size=D)) * 999.0 + 10.0)


def _ctx(env=ENV, n=32, T=8, **envvars):
    old = {k: os.environ.get(k) for k in envvars}
    os.environ.update({k: str(v) for k, v in envvars.items()})
    try:
        ctx, cfg, inst = make_ctx(env, n, T)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return ctx, cfg, inst


def _state(ctx, P):
    return [(ctx.params_get(p).copy(), *[np.copy(x) for x in ctx.adam_get(p)]) for p in range(P)]


def _schedule(ctx, P, seed=3):
    import torch
    rng = np.random.default_rng(seed)
    sh, pe = [], []
    for p in range(P):
        R = ctx.layout[p]["C"] * ctx.cfg.frag_len
        nb = R // 128
        sh.append(torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda())
        pe.append(torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(10)]).astype(np.int32)).cuda())
    return sh, pe


def _prepare(ctx, cfg, inst, seed=7):
    rng = np.random.default_rng(seed)
    params = init_params(ctx, cfg, seed, head_scale=1.0)
    run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), cfg.frag_len)


def test_failed_fused_update_leaves_state_unchanged():
    from ddrl_amd.native import DdrlError
    ctx, cfg, inst = _ctx(DDRL_TEST_FAIL_STEP=5)
    _prepare(ctx, cfg, inst)
    P = cfg.n_policies
    # two healthy-looking Adam steps first: the beta powers / moments are no longer the init values
    ctx.adam_set(0, *[np.full(ctx.n_params[0], 1e-3, np.float32)] * 2, 0.9 ** 3, 0.999 ** 3)
    before = _state(ctx, P)
    sh, pe = _schedule(ctx, P)
    ctx.ppo_update((1 << P) - 1, sh, pe, [0.2] * P)
    with pytest.raises(DdrlError, match="as before the call"):
        ctx.ppo_stats(0, 4)
    after = _state(ctx, P)
    for b, a in zip(before, after):
        for x, y in zip(b, a):
            np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    ctx.close()
    # a healthy context of the same data runs the same update normally
    ok, cfg2, inst2 = _ctx()
    _prepare(ok, cfg2, inst2)
    sh, pe = _schedule(ok, P)
    ok.ppo_update((1 << P) - 1, sh, pe, [0.2] * P, max_steps=8)
    st = ok.ppo_stats(0, 8)
    assert np.isfinite(st).all()
    ok.close()


def test_atomic_exchange_matches_default_protocol_bit_for_bit():
    P = 4
    res = []
    for env in ({}, {"DDRL_XCHG": "atomic"}):
        ctx, cfg, inst = _ctx(**env)
        _prepare(ctx, cfg, inst)
        sh, pe = _schedule(ctx, P)
        ctx.ppo_update((1 << P) - 1, sh, pe, [0.2] * P)   # the whole 10-epoch schedule (20 steps)
        res.append((_state(ctx, P), ctx.ppo_stats(0, 20)))
        ctx.close()
    (sa, st_a), (sb, st_b) = res
    for x, y in zip(sa, sb):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(np.asarray(u), np.asarray(v))
    np.testing.assert_array_equal(st_a, st_b)


def test_short_launches_match_atomic_protocol_bit_for_bit():
    """Consecutive fused launches of 1, 2, 3 and 5 steps: every launch clears the outboxes and
    restarts the one-bit LSB tags at step 0, so the first steps of each launch (zero words
    must fail the tag) and a tag's return after two steps are exercised launch after launch.
    The atomic protocol sums the same LSB-replaced partials through {value, tag} pairs."""
    P = 4
    res = []
    for env in ({}, {"DDRL_XCHG": "atomic"}):
        ctx, cfg, inst = _ctx(**env)
        _prepare(ctx, cfg, inst)
        st = []
        for i, k in enumerate((1, 2, 3, 5)):
            sh, pe = _schedule(ctx, P, seed=100 + i)
            ctx.ppo_update((1 << P) - 1, sh, pe, [0.2] * P, max_steps=k)
            st.append(ctx.ppo_stats(0, k))
        res.append((_state(ctx, P), st))
        ctx.close()
    (sa, st_a), (sb, st_b) = res
    for x, y in zip(sa, sb):
        for u, v in zip(x, y):
            np.testing.assert_array_equal(np.asarray(u), np.asarray(v))
    for a, b in zip(st_a, st_b):
        np.testing.assert_array_equal(a, b)


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


def test_failed_native_ddp_loop_leaves_state_unchanged(pg1):
    import torch
    from ddrl_amd.ddp import Comm, NativeDataParallelLearner
    from ddrl_amd.native import DdrlError
    ctx, cfg, inst = _ctx("QuantrupedMultiEnv_SharedDecentral", 32, 4, DDRL_TEST_FAIL_STEP=0)
    _prepare(ctx, cfg, inst)
    before = _state(ctx, 1)
    nat = NativeDataParallelLearner(ctx, Comm("cpu"), 0, 128, "split")
    from ddrl_amd.ddp import native_comm_init
    native_comm_init(ctx, Comm("cpu"))
    R = ctx.layout[0]["C"] * cfg.frag_len
    shuffle, perms = nat.schedule(np.random.default_rng(1), R, 2)
    with pytest.raises(DdrlError, match="as before the call"):
        nat.learn(torch.from_numpy(shuffle).cuda(), perms, 0.2)
    after = _state(ctx, 1)
    for x, y in zip(before[0], after[0]):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    ctx.close()
