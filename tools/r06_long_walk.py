"""r06 diagnostic: the Local tie-following comparison of tests/test_gpu_longhorizon.py carried past
one epoch, for one policy (GPU box, repo root):

    python tools/r06_long_walk.py [policy] [steps]      # default policy 0, 64,000 steps (the iteration)
    python tools/r06_long_walk.py -1 25600              # C4's shared policy, one epoch
    python tools/r06_long_walk.py -2 12800              # C5's GraphNet, one epoch of one-launch steps

The bench configuration (4096 envs x T = 200, the test's seeds), policy `policy`: HIP walked one
step at a time (ddrl_ppo_update_from) beside the fp64 trajectory that follows its clip outcomes,
and the numpy fp32 oracle walked the same way beside its own; distances printed at every horizon
and progress every 2,000 steps."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def setup_c4():
    """C4 as tests/test_gpu_fullsize_shared.py's quarter-epoch test (4096 envs, its seeds)."""
    from oracle import ddrl_oracle as O
    from tests.test_gpu_fullsize_shared import C4_ENV, C4_N, _ffn_batch, _rollout
    ctx, cfg, params, _, syn = _rollout(C4_ENV, C4_N, 13, False)
    del syn
    rec = ctx.records_get(0)
    d, A = cfg.obs_dim[0], cfg.act_dim
    batch = _ffn_batch(rec, ctx.layout[0], d, A, ctx.adv_norm_get(0))
    sh, pe = O.sgd_schedule(np.random.default_rng(44), rec.shape[0], 128, 10)
    return ctx, params, O.ffn_param_shapes(d, 2 * A), batch, sh, pe


def setup_c5():
    """C5 as tests/test_gpu_fullsize_shared.py's 1,000-step test (2048 envs, its seeds)."""
    from oracle import ddrl_oracle as O
    from tests.gpu_harness import GNN_ENV
    from tests.test_gpu_fullsize_shared import C5_N, _gnn_batch, _rollout, _schedule
    ctx, cfg, params, _, syn = _rollout(GNN_ENV, C5_N, 17, True)
    del syn
    rec = ctx.records_get(0)
    sh, pe = _schedule(rec.shape[0], 8)
    return ctx, params, O.gnn_param_shapes(4), _gnn_batch(rec, ctx.layout[0], ctx.adv_norm_get(0)), sh.numpy(), pe.numpy()


def main(q=0, steps=64000):
    """q = Local policy q; q = -1: C4's shared policy; q = -2: C5's GraphNet."""
    import torch
    from oracle import ddrl_oracle as O
    from ddrl_amd.synthetic import SyntheticRollout
    from tests.gpu_harness import HipLockstep, NumpyLockstep, init_params, make_ctx, tie_following_trajectory
    from tests.test_gpu_longhorizon import N_ENVS, T, _batch
    model = "gnn" if q == -2 else "ffn"
    if q < 0:
        ctx, p0, shapes, batch, sh, pe = setup_c4() if q == -1 else setup_c5()
        params, q = [p0], 0
    else:
        ctx, cfg, _ = make_ctx("QuantrupedMultiEnv_Local", N_ENVS, T)
        params = init_params(ctx, cfg, 21, head_scale=1.0)
        syn = SyntheticRollout(N_ENVS, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=3)
        ctx.observe(syn.obs[0])
        ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, syn.dones_for_fragment(), syn.actions)
        ctx.gae()
        ctx.synchronize()
        del syn
        R = T * ctx.layout[0]["C"]
        sched = [O.sgd_schedule(np.random.default_rng(40 + p), R, 128, 10) for p in range(4)]
        A = cfg.act_dim
        shapes = O.ffn_param_shapes(cfg.obs_dim[q], 2 * A)
        batch = _batch(ctx.records_get(q), ctx.layout[q], cfg.obs_dim[q], A, ctx.adv_norm_get(q))
        sh, pe = sched[q]
    horizons = sorted({h for h in (100, 400, 1000, 1600, 2000, 3200, 4000, 6400, 9600, 12800, 19200, 25600, 32000, 44800, 64000) if h <= steps} | {steps})
    t0 = time.time()

    class Progress:
        """Wraps an implementation: a progress line every 2,000 steps (the box's hang detector)."""
        def __init__(self, impl, tag):
            self.impl, self.tag = impl, tag
            self.snaps = impl.snaps

        def grad(self, rows):
            return self.impl.grad(rows)

        def step(self, k):
            self.impl.step(k)
            if (k + 1) % (200 if model == "gnn" else 2000) == 0:
                print(f"{self.tag}: step {k + 1} ({time.time() - t0:.0f} s)", flush=True)

        def theta(self):
            return self.impl.theta()

    # past the first epoch most steps differ by more than the search threshold with no flip to
    # explain them (smooth drift): a small search keeps the walk affordable
    search = dict(pool=16, max_flips=2)
    npl = NumpyLockstep(params[q], shapes, batch, sh, pe, 0.2, model=model)
    m32 = []
    tf32, _, ties32 = tie_following_trajectory(None, q, params[q], shapes, batch, sh, pe, 0.2, steps, horizons,
                                               impl=Progress(npl, "numpy"), missed=m32, model=model, **search)
    for h in horizons:
        print(f"numpy H={h}: |numpy fp32 - fp64 following numpy| {np.abs(npl.snaps[h] - tf32[h]).max():.3g}", flush=True)
    hip = HipLockstep(ctx, q, O.pack(params[q], shapes), sh, pe, 0.2)
    mh = []
    tf, _, ties = tie_following_trajectory(ctx, q, params[q], shapes, batch, sh, pe, 0.2, steps, horizons,
                                           impl=Progress(hip, "HIP"), missed=mh, model=model, **search)
    print(f"policy {q}: flips HIP {len(ties)}, numpy {len(ties32)}; unexplained steps HIP {len(mh)} "
          f"(first {mh[0][0] if mh else '-'}), numpy {len(m32)} (first {m32[0][0] if m32 else '-'})", flush=True)
    for h in horizons:
        eh = np.abs(hip.snaps[h] - tf[h]).max()
        en = np.abs(npl.snaps[h] - tf32[h]).max()
        moved = np.abs(tf[h] - O.pack(params[q], shapes)).max()
        print(f"H={h}: |HIP - fp64 following HIP| {eh:.3g}, |numpy fp32 - fp64 following numpy| {en:.3g}, "
              f"HIP / numpy {eh / en if en else float('inf'):.2f}; max |theta - theta0| {moved:.3g}", flush=True)
    ctx.close()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
