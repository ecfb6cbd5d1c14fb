"""Peer mode: the shared-policy minibatch SGD of two ranks as one fused update
split across two contexts (ddrl_ppo_update_peer).

SharedDecentral ("policy_legs" on all four legs,
quantruped_singleDecentralizedController_environments.py:21-48), "split" semantics: the
reference's 128-row minibatch, 64 rows from each rank's shard.  Rank r's fused launch runs row
half r of every minibatch and swaps its partial gradients with the peer launch every step
through shared outboxes (LSB-tagged quads with system-scope stores and loads, ppo_ffn_peer.hip);
both then run the same clip + tf1 Adam.
Rehearsed here as two contexts of one process on one GPU, each on its own stream, so the two
persistent launches run side by side (the pool gives one GPU: the xGMI path is not exercised).

Checks: both ranks' weights, Adam moments, beta powers and learner statistics are bit-identical
to each other AND to ONE fused launch (ddrl_ppo_update) over the union batch whose minibatch b is
[rank 0's 64 rows | rank 1's 64 rows] -- the row halves of that launch do exactly the two ranks'
arithmetic on the same LSB-replaced partials.  Two consecutive updates keep the ranks' launch
tags and global step count (the quads' tag bit) in lockstep.  A rank whose peer never launches
abandons its waits at the 3 s bound: the call raises and its state is restored.  Then the same as
two processes sharing the GPU (IPC-mapped outboxes): the trainer's PeerLearner ("ddp_loop":
"peer") against the per-step all-reduce learner.
"""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import init_params, make_ctx, run_rollout

pytestmark = pytest.mark.gpu
ENV = "QuantrupedMultiEnv_SharedDecentral"
N_ENVS, T = 32, 8          # 1,024 rows per rank, 2,048 in the union batch


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _filt(D, rng):
    return (1000.0, rng.normal(size=D) * 0.3, np.abs(rng.normal(size=D)) * 999.0 + 10.0)


def _rank_records(seed):
    ctx, cfg, inst = make_ctx(ENV, N_ENVS, T)
    params = init_params(ctx, cfg, 7, head_scale=1.0)      # the same weights on both ranks
    rng = np.random.default_rng(seed)
    run_rollout(ctx, cfg, inst, params, rng, _filt(cfg.obs_full_dim, rng), T)
    return ctx, cfg, ctx.records_get(0)


def _state(ctx):
    m, v, b1, b2 = ctx.adam_get(0)
    return [ctx.params_get(0).copy(), m.copy(), v.copy(), np.float32(b1), np.float32(b2)]


@pytest.fixture(scope="module")
def setup():
    import torch
    ranks = [_rank_records(100 + r) for r in range(2)]
    cfg = ranks[0][1]
    lay = ranks[0][0].layout[0]
    R = ranks[0][2].shape[0]
    nb = R // 64
    # StandardizeFields over the union batch (what the trainer all-reduces)
    adv = np.concatenate([r[2][:, lay["adv"]] for r in ranks])
    _, mean, std = O.standardize(adv)
    norm = (float(mean), float(max(np.float32(1e-4), std)))
    rng = np.random.default_rng(5)
    sh = [rng.permutation(R).astype(np.int32) for _ in range(2)]
    pe = np.stack([rng.permutation(nb) for _ in range(cfg.num_sgd_iter)]).astype(np.int32)
    # the union launch: records rank-major, minibatch slot b = [rank 0 rows | rank 1 rows + R]
    usch = np.empty(nb * 128, np.int32)
    for b in range(nb):
        usch[b * 128:b * 128 + 64] = sh[0][b * 64:(b + 1) * 64]
        usch[b * 128 + 64:(b + 1) * 128] = R + sh[1][b * 64:(b + 1) * 64]
    uctx, ucfg, _ = make_ctx(ENV, 2 * N_ENVS, T)
    uctx.params_set(0, ranks[0][0].params_get(0))
    uctx.records_set(0, np.concatenate([r[2] for r in ranks]))
    theta0 = ranks[0][0].params_get(0).copy()
    yield dict(ranks=ranks, cfg=cfg, norm=norm, sh=sh, pe=pe, usch=usch, uctx=uctx, theta0=theta0, nb=nb)
    uctx.close()
    for ctx, _, _ in ranks:
        ctx.close()
    torch.cuda.synchronize()


def _reset(ctx, theta0, norm):
    n = theta0.size
    ctx.params_set(0, theta0)
    ctx.adam_set(0, np.zeros(n, np.float32), np.zeros(n, np.float32), 0.9, 0.999)
    ctx.adv_norm_set(0, *norm)


def test_peer_update_equals_union_fused_update_bit_for_bit(setup):
    import torch
    S = setup
    ctxs = [r[0] for r in S["ranks"]]
    nb, steps = S["nb"], S["cfg"].num_sgd_iter * S["nb"]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    pe_d, sh_d = dev(S["pe"]), [dev(s) for s in S["sh"]]
    # reference: one fused launch over the union batch, twice (two iterations' updates)
    u = S["uctx"]
    _reset(u, S["theta0"], S["norm"])
    u.ppo_update(1, [dev(S["usch"])], [pe_d], [0.2])
    u.synchronize()
    ref1 = (_state(u), u.ppo_stats(0, steps))
    u.ppo_update(1, [dev(S["usch"])], [pe_d], [0.3], max_steps=37)
    u.synchronize()
    ref2 = (_state(u), u.ppo_stats(0, 37))
    # peer mode: each context on its own stream, both launches enqueued before either is waited for
    streams = [torch.cuda.Stream() for _ in range(2)]
    torch.cuda.synchronize()
    gx, _ = ctxs[0].peer_alloc()
    for r, ctx in enumerate(ctxs):
        _reset(ctx, S["theta0"], S["norm"])
        ctx.set_stream(streams[r].cuda_stream)
        ctx.peer_attach(gx, r, 2)
    for kl, ms, ref in ((0.2, -1, ref1), (0.3, 37, ref2)):
        for r, ctx in enumerate(ctxs):
            ctx.ppo_update_peer(0, sh_d[r], pe_d, kl, max_steps=ms)
        for ctx in ctxs:
            ctx.synchronize()
        n = steps if ms < 0 else ms
        got = [(_state(ctx), ctx.ppo_stats(0, n)) for ctx in ctxs]
        for st, stats in got:
            for x, y in zip(st, ref[0]):
                np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
            np.testing.assert_array_equal(stats, ref[1])
    assert not np.array_equal(got[0][0][0], S["theta0"])
    for r, ctx in enumerate(ctxs):
        ctx.set_stream(torch.cuda.current_stream().cuda_stream)


def test_peer_update_without_its_peer_fails_and_restores(setup):
    import torch
    from ddrl_amd.native import DdrlError
    S = setup
    ctx = S["ranks"][0][0]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    _reset(ctx, S["theta0"], S["norm"])
    before = _state(ctx)
    gx, _ = ctx.peer_alloc()
    ctx.peer_attach(gx, 0, 2)
    ctx.ppo_update_peer(0, dev(S["sh"][0]), dev(S["pe"]), 0.2, max_steps=3)
    with pytest.raises(DdrlError, match="as before the call") as ei:
        ctx.synchronize()
    assert "ddrl_peer_attach again" in str(ei.value)
    for x, y in zip(before, _state(ctx)):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    # the failed launch may have left partly written outboxes, so the context is
    # detached -- a retry without re-attaching is refused before any launch, the state unchanged
    with pytest.raises(DdrlError, match="no peer"):
        ctx.ppo_update_peer(0, dev(S["sh"][0]), dev(S["pe"]), 0.2, max_steps=3)
    for x, y in zip(before, _state(ctx)):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
    # re-attaching (rank 0 clears the outboxes) is accepted again
    ctx.peer_attach(gx, 0, 2)
    ctx.synchronize()


def _peer_rank(rank, world, port, out_dir):
    import os
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)          # both ranks share the one GPU of the box
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ddrl_amd.trainer import PPOTrainer
    out = {}
    for loop in ("peer", "python"):
        tr = PPOTrainer({"env": ENV, "rollout_fragment_length": 8, "parallel": "ddp", "ddp_loop": loop,
                         "observation_filter": "MeanStdFilter"}, n_envs=32, seed=5)
        pid = tr.policy_ids[0]
        for it in range(2):
            r = tr.train()
            out[f"{loop}_w{it}"] = tr.get_weights()[pid]
            out[f"{loop}_kl{it}"] = np.array([r["info"]["learner"][pid]["kl"]])
            out[f"{loop}_loss{it}"] = np.array([r["info"]["learner"][pid]["total_loss"]])
        tr.stop()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), **out)
    dist.destroy_process_group()


def test_peer_learner_two_processes_match_data_parallel_learner():
    """Two processes on the box's GPU (the outboxes shared by IPC handle, handed over with a gloo
    broadcast), PPOTrainer "ddp_loop": "peer": both ranks' weights bit-identical after each of two
    iterations, and within the fused path's bar of the per-step all-reduce learner ("python")
    on the same rollouts and schedule (the fused exchange's LSB tags are the only difference)."""
    import os
    import socket
    import tempfile
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tempfile.mkdtemp()
    mp.spawn(_peer_rank, args=(2, port, out), nprocs=2, join=True)
    a, b = (np.load(os.path.join(out, f"r{r}.npz")) for r in range(2))
    for it in range(2):
        np.testing.assert_array_equal(a[f"peer_w{it}"], b[f"peer_w{it}"])
        assert a[f"peer_kl{it}"][0] == b[f"peer_kl{it}"][0]
        ref, got = a[f"python_w{it}"].astype(np.float64), a[f"peer_w{it}"].astype(np.float64)
        diff = np.abs(got - ref)
        frac = float(np.mean(diff <= 1e-5 + 1e-5 * np.abs(ref)))
        print(f"\niteration {it}: peer vs per-step all-reduce learner: max |diff| {diff.max():.3g}, "
              f"{frac:.5f} within 1e-5 + 1e-5 |w|; kl {a[f'peer_kl{it}'][0]:.6g} vs {a[f'python_kl{it}'][0]:.6g}")
        assert frac >= 0.999 and diff.max() <= 2 * 3e-4 * 8 + 1e-5
        np.testing.assert_allclose(a[f"peer_kl{it}"], a[f"python_kl{it}"], rtol=1e-3, atol=1e-7)
    assert not np.array_equal(a["peer_w1"], a["peer_w0"])


def test_peer_mode_argument_checks(setup):
    """The C-ABI refuses what peer mode does not support, before anything is launched."""
    import torch
    from ddrl_amd.native import DdrlError
    S = setup
    ctx = S["ranks"][0][0]
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    fresh, _, _ = make_ctx(ENV, N_ENVS, T)
    try:
        with pytest.raises(DdrlError, match="no peer"):
            fresh.ppo_update_peer(0, dev(S["sh"][0]), dev(S["pe"]), 0.2)
        gx, _ = ctx.peer_alloc()
        with pytest.raises(DdrlError, match="exactly two ranks"):
            fresh.peer_attach(gx, 0, 3)
        with pytest.raises(DdrlError, match="exactly two ranks"):
            fresh.peer_attach(gx, 2, 2)
        fresh.peer_attach(gx, 0, 2)
        too_many = np.zeros((10, S["nb"] + 1), np.int32)
        with pytest.raises(DdrlError, match="exceed this rank's train batch"):
            fresh.ppo_update_peer(0, dev(np.zeros(64 * (S["nb"] + 1), np.int32)), dev(too_many), 0.2)
        with pytest.raises(DdrlError, match="bad policy id"):
            fresh.ppo_update_peer(1, dev(S["sh"][0]), dev(S["pe"]), 0.2)
    finally:
        fresh.close()
