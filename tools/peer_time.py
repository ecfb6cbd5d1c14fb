"""Peer mode timing on one GPU ("Peer mode"): C4 (SharedDecentral, 4096 envs
x T = 200) as two ranks of 2048 envs each, two contexts of one process on two streams, against
one fused launch over the union batch and against one rank's half-size fused update.

Prints, per variant, microseconds per minibatch step over `--steps` steps (wall clock around
the launch, after a warm-up launch): the concurrent peer launches exchange their partials
through fine-grained device memory with system-scope atomics on the same GPU, so this measures
the peer protocol's cost without the xGMI hop (unmeasured: the pool gives one GPU).
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddrl_amd import native as N
from ddrl_amd.spec import make_cfg
from ddrl_amd.synthetic import SyntheticRollout

ENV, T = "QuantrupedMultiEnv_SharedDecentral", 200


def rollout(n, seed, stream, atomic=False):
    cfg, _ = make_cfg(ENV, n, T)
    if atomic:
        os.environ["DDRL_XCHG"] = "atomic"   # read at context creation
    ctx = N.Context(cfg, 0, stream)
    os.environ.pop("DDRL_XCHG", None)
    rng = np.random.default_rng(7)           # the same weights in every context
    ctx.params_set(0, (rng.normal(size=ctx.n_params[0]) * 0.05).astype(np.float32))
    syn = SyntheticRollout(n, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=seed)
    done = syn.dones_for_fragment()
    torch.cuda.synchronize()   # the inputs are made on torch's stream, the context may use another
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, done, syn.actions)
    ctx.gae()
    ctx.synchronize()
    return ctx, cfg


def timed(fn, sync):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    sync()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=4000)
    a = ap.parse_args()
    n2 = a.envs // 2
    streams = [torch.cuda.Stream() for _ in range(2)]
    ranks = [rollout(n2, 11 + r, streams[r].cuda_stream) for r in range(2)]
    R = ranks[0][0].layout[0]["C"] * T
    nb = R // 64
    rng = np.random.default_rng(3)
    sh = [torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda() for _ in range(2)]
    pe = torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(10)]).astype(np.int32)).cuda()
    # one fused launch over the union batch (default exchange protocol, and the atomic one the
    # peer launches use)
    u, _ = rollout(a.envs, 11, torch.cuda.current_stream().cuda_stream)
    ush = torch.stack([sh[0].view(nb, 64), sh[1].view(nb, 64) + R], 1).reshape(-1).contiguous()
    ua, _ = rollout(a.envs, 11, torch.cuda.current_stream().cuda_stream, atomic=True)
    res = {}
    for name in ("union", "union_warm"):
        res[name] = timed(lambda: u.ppo_update(1, [ush], [pe], [0.2], max_steps=a.steps), u.synchronize)
    for name in ("union_atomic", "union_atomic_warm"):
        res[name] = timed(lambda: ua.ppo_update(1, [ush], [pe], [0.2], max_steps=a.steps), ua.synchronize)
    # one rank's half-size batch alone (128-row minibatches over 2048 envs)
    c0 = ranks[0][0]
    pe_h = torch.from_numpy(np.stack([rng.permutation(R // 128) for _ in range(10)]).astype(np.int32)).cuda()
    for name in ("half", "half_warm"):
        res[name] = timed(lambda: c0.ppo_update(1, [sh[0]], [pe_h], [0.2], max_steps=a.steps), c0.synchronize)
    # peer pair, both ranks from the same weights and a cleared Adam state
    th0 = u.params_get(0)
    for ctx, _ in ranks:
        ctx.params_set(0, th0)
        ctx.adam_set(0, np.zeros(th0.size, np.float32), np.zeros(th0.size, np.float32), 0.9, 0.999)
    gx, _ = ranks[0][0].peer_alloc()
    for r, (ctx, _) in enumerate(ranks):
        ctx.peer_attach(gx, r, 2)

    def peer():
        for r, (ctx, _) in enumerate(ranks):
            ctx.ppo_update_peer(0, sh[r], pe, 0.2, max_steps=a.steps)

    def sync_both():
        for ctx, _ in ranks:
            ctx.synchronize()
    for name in ("peer", "peer_warm"):
        res[name] = timed(peer, sync_both)
    th = [ctx.params_get(0) for ctx, _ in ranks]
    same = bool(np.array_equal(th[0], th[1]))
    for k in ("union_warm", "union_atomic_warm", "half_warm", "peer_warm"):
        print(f"{k:18s} {res[k] * 1e6 / a.steps:8.3f} us/step over {a.steps} steps", flush=True)
    print(f"peer ranks bit-identical: {same}", flush=True)
    for ctx, _ in ranks:
        ctx.close()
    u.close()
    ua.close()


if __name__ == "__main__":
    main()
