"""why does the HIP C4 fused update leave the fp32 family before H = 1,600?

Runs on the GPU box (one process).  Builds the C4 full-size rollout exactly as
tests/test_gpu_fullsize_shared.py does (4096 envs, T = 200, seed 13, schedule rng 44), then:

  A  HIP default fused launch (row split, LSB-tagged exchange): max |theta - fp64| after every
     H = 1..HMAX steps (one launch per H from the same start);
  B  the same with DDRL_UPDATE_SPLIT=1 (no row split, so no LSB replacement);
  C  the one-rank data-parallel loop (ddrl_ppo_grad + ddrl_ppo_apply per step: the pair path,
     partials added untouched);
  D  numpy oracles: fp64, fp32, fp32 with the LSB replacement emulated (each 64-row half's
     partial gradient has its mantissa LSB forced to the step's tag bit before the add), fp32
     with Adam's sqrt / rcp perturbed by one ulp, fp32 with the step's clip scale off by one ulp;
  E  local error: from the numpy fp32 state after k steps, one HIP step vs one numpy step vs the
     fp64 step from the same state, k = 0, 50, ...;
  F  at the first step where HIP leaves fp64 (> 1e-5), the rows of that minibatch whose clip
     branch differs between HIP's state and the fp64 trajectory's state, with their margins.

Writes gpurun_out/r06/c4diag.npz and prints a summary.  Test infrastructure: imports the oracle.
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import ddrl_oracle as O  # noqa: E402

T, NENV, HMAX = 200, 4096, int(os.environ.get("HMAX", "1600"))
ENV = "QuantrupedMultiEnv_SharedDecentral"
OUT = os.path.join(ROOT, "gpurun_out", "r06")
t_start = time.time()


def log(*a):
    print(f"[{time.time() - t_start:7.1f}s]", *a, flush=True)


# ------------------------------------------------------------------ oracle single step
def lx(x, bit):
    u = np.asarray(x, np.float32).view(np.uint32)
    return ((u & np.uint32(0xFFFFFFFE)) | np.uint32(bit)).view(np.float32)


def ulp_jitter(x, rng):
    x = np.asarray(x, np.float32)
    up = rng.random(x.shape) < 0.5
    return np.where(up, np.nextafter(x, np.float32(np.inf)), np.nextafter(x, np.float32(-np.inf))).astype(np.float32)


class State:
    def __init__(self, mod, theta, n):
        self.mod = mod
        F = mod.F32
        self.theta = np.asarray(theta, F).copy()
        self.adam = mod.Adam(n)

    def copy(self):
        s = State.__new__(State)
        s.mod = self.mod
        s.theta = self.theta.copy()
        a = self.mod.Adam(self.theta.size)
        a.m, a.v, a.b1p, a.b2p = self.adam.m.copy(), self.adam.v.copy(), self.adam.b1p, self.adam.b2p
        s.adam = a
        return s


def one_step(st, shapes, batch, rows, kl, mode="plain", k=0, rng=None):
    """One minibatch step of ddrl_oracle.ppo_update on state st (in place).  mode: plain | lx |
    adamulp | clipulp."""
    M = st.mod
    F = M.F32
    p = M.unpack(st.theta, shapes)
    logits, value, cache = M.ffn_forward(p, batch["obs"][rows])
    dlogits, dvalue, stats = M.ppo_loss_rows(logits, value, batch["actions"][rows], batch["logits"][rows],
                                             batch["logp"][rows], batch["vf_preds"][rows], batch["adv"][rows],
                                             batch["vt"][rows], F(kl))
    if mode == "lx":
        bit = ((k >> 1) & 1) ^ 1
        h = [M.ffn_backward(p, tuple(c[s] for c in cache), dlogits[s], dvalue[s])
             for s in (slice(0, 64), slice(64, 128))]
        g = {n: (lx(h[0][n], bit) + lx(h[1][n], bit)).astype(F) for n, _ in shapes}
    else:
        g = M.ffn_backward(p, cache, dlogits, dvalue)
    glist = [g[n] for n, _ in shapes]
    clipped, gn = M.clip_by_global_norm(glist)
    if mode == "clipulp":
        clipped = [np.asarray(c, F) for c in clipped]
        scale = np.float32(0.5) * min(np.float32(1.0) / gn, np.float32(2.0))
        s2 = ulp_jitter(np.array([scale], np.float32), rng)[0]
        clipped = [(c / scale * s2).astype(F) for c in clipped]
    flat = np.concatenate([c.reshape(-1) for c in clipped])
    if mode == "adamulp":
        a = st.adam
        one = F(1.0)
        alpha = a.lr * np.sqrt(one - a.b2p) / (one - a.b1p)
        a.m = a.m + (flat - a.m) * (one - a.b1)
        a.v = a.v + (flat * flat - a.v) * (one - a.b2)
        den = ulp_jitter(np.sqrt(a.v), rng) + a.eps
        st.theta = (st.theta - (a.m * alpha) * ulp_jitter(one / den, rng)).astype(F)
        a.b1p = F(a.b1p * a.b1)
        a.b2p = F(a.b2p * a.b2)
    else:
        st.theta = st.adam.apply(st.theta, flat)
    stats["grad_gnorm"] = float(gn)
    return stats


def row_branches(mod, theta, shapes, batch, rows, clip=0.2, vclip=10.0):
    """fp64 per-row clip state: (policy gradient active, value branch code, policy margin, value margin)."""
    p = O.unpack(theta, shapes) if mod is None else mod.unpack(theta, shapes)
    p = {k: v.astype(np.float64) for k, v in p.items()}
    x = batch["obs"][rows].astype(np.float64)
    h1 = np.tanh(x @ p["fc_1/kernel"] + p["fc_1/bias"])
    h2 = np.tanh(h1 @ p["fc_2/kernel"] + p["fc_2/bias"])
    logits = h2 @ p["fc_out/kernel"] + p["fc_out/bias"]
    g1 = np.tanh(x @ p["fc_value_1/kernel"] + p["fc_value_1/bias"])
    g2 = np.tanh(g1 @ p["fc_value_2/kernel"] + p["fc_value_2/bias"])
    value = (g2 @ p["value_out/kernel"] + p["value_out/bias"])[:, 0]
    A = logits.shape[1] // 2
    mean, ls = logits[:, :A], logits[:, A:]
    z = (batch["actions"][rows] - mean) / np.exp(ls)
    logp = -0.5 * np.sum(z * z, 1) - 0.5 * np.log(2 * np.pi) * A - np.sum(ls, 1)
    ratio = np.exp(logp - batch["logp"][rows].astype(np.float64))
    adv = batch["adv"][rows].astype(np.float64)
    lo, hi = 1 - clip, 1 + clip
    active = np.where(adv >= 0, ratio <= hi, ratio >= lo)
    pm = np.where(adv >= 0, ratio - hi, lo - ratio)
    vf_old, vt = batch["vf_preds"][rows].astype(np.float64), batch["vt"][rows].astype(np.float64)
    dv = value - vf_old
    vcl = vf_old + np.clip(dv, -vclip, vclip)
    vf1, vf2 = (value - vt) ** 2, (vcl - vt) ** 2
    vcode = np.where(vf1 >= vf2, 0, np.where(np.abs(dv) <= vclip, 1, 2))
    vm = np.minimum(np.abs(np.abs(dv) - vclip), np.abs(vf1 - vf2))
    return active, vcode, pm, vm, ratio, dv


def main():
    import torch
    from ddrl_amd import native as N
    from ddrl_amd.spec import make_cfg
    from ddrl_amd.synthetic import SyntheticRollout
    from tests.gpu_harness import init_params, make_ctx

    os.makedirs(OUT, exist_ok=True)
    ctx, cfg, inst = make_ctx(ENV, NENV, T)
    params = init_params(ctx, cfg, 13, head_scale=1.0)[0]
    syn = SyntheticRollout(NENV, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=13)
    done = syn.dones_for_fragment()
    ctx.observe(syn.obs[0])
    ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, done, syn.actions)
    ctx.gae()
    ctx.synchronize()
    del syn
    rec = ctx.records_get(0)
    lay = ctx.layout[0]
    d, A = cfg.obs_dim[0], cfg.act_dim
    mean, den = ctx.adv_norm_get(0)
    batch = dict(obs=rec[:, :d], actions=rec[:, lay["act"]:lay["act"] + A],
                 logits=rec[:, lay["logit"]:lay["logit"] + 2 * A], logp=rec[:, lay["logp"]],
                 vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                 vt=rec[:, lay["vt"]])
    shapes = O.ffn_param_shapes(d, 2 * A)
    theta0 = O.pack(params, shapes)
    n = theta0.size
    R = rec.shape[0]
    sh, pe = O.sgd_schedule(np.random.default_rng(44), R, 128, 10)
    nb = R // 128
    assert HMAX < nb
    rows_of = lambda k: sh[pe[0, k] * 128:(pe[0, k] + 1) * 128]
    log(f"rollout done: R={R}, n_params={n}, adv norm {mean:.6g} {den:.6g}")

    # ---------------------------------------------------------------- D: oracle trajectories
    O64 = O.with_dtype(np.float64)
    trajs = {}
    ckpt = {}
    stats = {}
    for name, mod, mode in [("fp64", O64, "plain"), ("fp32", O, "plain"), ("lx32", O, "lx"),
                            ("adamulp32", O, "adamulp"), ("clipulp32", O, "clipulp")]:
        st = State(mod, theta0, n)
        rng = np.random.default_rng(7)
        th = np.empty((HMAX + 1, n), np.float64)
        th[0] = theta0
        sts = []
        for k in range(HMAX):
            if name == "fp32" and k % 50 == 0:
                ckpt[k] = st.copy()
            sts.append(one_step(st, shapes, batch, rows_of(k), 0.2, mode, k, rng))
            th[k + 1] = st.theta
        trajs[name] = th
        stats[name] = sts
        log(f"oracle {name}: done")
    th64 = trajs["fp64"]

    def dev(th):
        return np.abs(th - th64).max(1)

    curves = {k: dev(v) for k, v in trajs.items() if k != "fp64"}

    # ---------------------------------------------------------------- A/B: HIP sweeps
    dsh = torch.from_numpy(sh).cuda()
    dpe = torch.from_numpy(pe).cuda()

    def reset(c, theta, m=None, v=None, b1p=0.9, b2p=0.999):
        c.params_set(0, np.asarray(theta, np.float32))
        c.adam_set(0, np.zeros(n, np.float32) if m is None else m, np.zeros(n, np.float32) if v is None else v,
                   b1p, b2p)

    def sweep(c, label):
        out = np.zeros(HMAX + 1)
        th_keep = {}
        for H in range(1, HMAX + 1):
            reset(c, theta0)
            c.ppo_update(1, [dsh], [dpe], [0.2], max_steps=H)
            c.synchronize()
            got = c.params_get(0).astype(np.float64)
            out[H] = np.abs(got - th64[H]).max()
            th_keep[H] = got
        log(f"HIP sweep {label}: done")
        return out, th_keep

    curves["hip"], th_hip = sweep(ctx, "default")
    st_hip = ctx.ppo_stats(0, HMAX).astype(np.float64)

    os.environ["DDRL_UPDATE_SPLIT"] = "1"
    ctx1 = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
    del os.environ["DDRL_UPDATE_SPLIT"]
    ctx1.records_set(0, rec)
    ctx1.adv_norm_set(0, mean, den)
    curves["hip_split1"], _ = sweep(ctx1, "split=1")
    ctx1.close()

    # ---------------------------------------------------------------- C: one-rank DP loop
    reset(ctx, theta0)
    gbuf = torch.zeros(n, device="cuda")
    dp = np.zeros(HMAX + 1)
    for k in range(HMAX):
        r = torch.from_numpy(np.ascontiguousarray(rows_of(k))).cuda()
        ctx.ppo_grad(0, r, 128, 0.2, gbuf, k)
        ctx.ppo_apply(0, gbuf)
        ctx.synchronize()
        dp[k + 1] = np.abs(ctx.params_get(0).astype(np.float64) - th64[k + 1]).max()
    curves["hip_dp"] = dp
    log("HIP data-parallel loop: done")

    # ---------------------------------------------------------------- summary of the curves
    def first_over(c, thr=1e-5):
        w = np.flatnonzero(c > thr)
        return int(w[0]) if w.size else -1

    print("\nfirst H with max|theta - fp64| > 1e-5, and the deviation at H = 100/400/800/1200/1600:")
    for k, c in curves.items():
        hs = [h for h in (100, 400, 800, 1200, 1600) if h <= HMAX]
        print(f"  {k:11s} first {first_over(c):5d}   " + "  ".join(f"{h}:{c[h]:.3g}" for h in hs))

    # ---------------------------------------------------------------- E: local error
    print("\nlocal error: one step from the numpy fp32 state after k steps (max |theta - fp64 step|, "
          "and relative to max|fp64 update|)")
    loc = []
    for k in sorted(ckpt):
        s32 = ckpt[k]
        s64 = State(O64, s32.theta.astype(np.float64), n)
        s64.adam.m, s64.adam.v = s32.adam.m.astype(np.float64), s32.adam.v.astype(np.float64)
        s64.adam.b1p, s64.adam.b2p = np.float64(s32.adam.b1p), np.float64(s32.adam.b2p)
        one_step(s64, shapes, batch, rows_of(k), 0.2)
        a = s32.copy()
        one_step(a, shapes, batch, rows_of(k), 0.2)
        b = s32.copy()
        one_step(b, shapes, batch, rows_of(k), 0.2, "lx", 0)
        pek = pe.copy()
        pek[0, 0] = pe[0, k]
        reset(ctx, s32.theta, s32.adam.m, s32.adam.v, float(s32.adam.b1p), float(s32.adam.b2p))
        ctx.ppo_update(1, [dsh], [torch.from_numpy(pek).cuda()], [0.2], max_steps=1)
        ctx.synchronize()
        hip = ctx.params_get(0).astype(np.float64)
        upd = np.abs(s64.theta - s32.theta).max()
        e = [np.abs(x - s64.theta).max() for x in (hip, a.theta, b.theta)]
        loc.append([k] + e + [upd])
        print(f"  k={k:5d}: HIP {e[0]:.3g}  fp32 {e[1]:.3g}  lx32 {e[2]:.3g}   (update {upd:.3g}; "
              f"HIP/fp32 {e[0] / max(e[1], 1e-30):.2f})")

    # ---------------------------------------------------------------- F: the first departure
    s_star = first_over(curves["hip"])
    flips = []
    if s_star > 0:
        k = s_star - 1   # the step (0-based) whose result first leaves fp64
        rows = rows_of(k)
        ah, vh, pmh, vmh, rh, dvh = row_branches(None, th_hip[k] if k > 0 else theta0, shapes, batch, rows)
        a6, v6, pm6, vm6, r6, dv6 = row_branches(None, th64[k], shapes, batch, rows)
        print(f"\nHIP leaves fp64 at H = {s_star}: dev {curves['hip'][s_star - 1]:.3g} -> {curves['hip'][s_star]:.3g}")
        for i in range(128):
            if ah[i] != a6[i] or vh[i] != v6[i]:
                flips.append((i, int(rows[i]), bool(ah[i]), bool(a6[i]), int(vh[i]), int(v6[i]), rh[i], r6[i]))
        print(f"  rows whose fp64-evaluated clip branch differs between HIP's state and fp64's state: {flips}")
        o = np.argsort(np.abs(pm6))[:5]
        print("  smallest policy-clip margins at fp64's state (row, ratio_fp64, ratio_at_HIP_state, adv): " +
              ", ".join(f"({i}, {r6[i]:.9f}, {rh[i]:.9f}, {batch['adv'][rows[i]]:.3g})" for i in o))
        o = np.argsort(vm6)[:3]
        print("  smallest value-clip margins (row, dv_fp64, dv_HIP): " +
              ", ".join(f"({i}, {dv6[i]:.6f}, {dvh[i]:.6f})" for i in o))
        # the same step from HIP's own state: HIP vs fp64 vs fp32
        reset(ctx, theta0)
        if k > 0:
            ctx.ppo_update(1, [dsh], [dpe], [0.2], max_steps=k)
        ctx.synchronize()
        _, _, b1p, b2p = ctx.adam_get(0)
        print(f"  HIP state at step {k} read back (beta powers {b1p}, {b2p})")
        # the fp32 trajectory's branches at that step, for the record
        a3, v3, pm3, _, r3, _ = row_branches(None, trajs["fp32"][k], shapes, batch, rows)
        print(f"  fp32 trajectory: rows whose branch differs from fp64's: "
              f"{[i for i in range(128) if a3[i] != a6[i] or v3[i] != v6[i]]}")

    # stats departure: first step where HIP's learner statistics leave fp64's by > 1e-4 rel
    keys = [(1, "policy_loss"), (2, "vf_loss"), (3, "kl"), (4, "entropy"), (6, "grad_gnorm")]
    for col, key in keys:
        ref = np.array([s[key] for s in stats["fp64"]])
        dv_ = np.abs(st_hip[:, col] - ref) / (np.abs(ref) + 1e-6)
        d32 = np.abs(np.array([s[key] for s in stats["fp32"]]) - ref) / (np.abs(ref) + 1e-6)
        print(f"  stat {key:12s}: first step HIP rel dev > 1e-4: {first_over(dv_, 1e-4)}; fp32: {first_over(d32, 1e-4)}")

    np.savez_compressed(os.path.join(OUT, "c4diag.npz"), **{f"curve_{k}": v for k, v in curves.items()},
                        local=np.array(loc), st_hip=st_hip,
                        st64=np.array([[s[k] for _, k in keys] for s in stats["fp64"]]))
    ctx.close()
    log("done")


if __name__ == "__main__":
    main()
