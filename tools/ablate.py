"""Ablation timing of the fused update kernel: builds diagnostic variants that each skip
one phase (results are wrong; only the per-step time matters) and reports us/step.

    python tools/ablate.py build [variants...]        # in the container (hipcc)
    python tools/ablate.py run [envs] [variants...]   # on the GPU box

A variant is a comma-separated list of macro definitions (`DDRL_ABL_NO_DW2`,
`DDRL_GX_ST=16,DDRL_GX_LD=16`); "" is the baseline build.
"""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
VARIANTS = ["", "DDRL_ABL_NO_DW2", "DDRL_ABL_NO_DW1", "DDRL_ABL_NO_L2BWD", "DDRL_ABL_NO_PREFETCH",
            "DDRL_ABL_NO_ADAM", "DDRL_ABL_NO_EXCHANGE", "DDRL_ABL_NO_HEADDPP", "DDRL_ABL_NO_TANH"]


def paths(v):
    from ddrl_amd import native as N
    d = os.path.dirname(N.LIB_PATH)
    tag = "".join(ch if ch.isalnum() else "_" for ch in v.replace("DDRL_ABL_", "").replace("DDRL_", "")).lower() or "base"
    return os.path.join(d, f"libddrl_hip_abl_{tag}.so"), os.path.join(d, f"_build_abl_{tag}")


def flags(v):
    return [f"-D{x}" for x in v.split(",") if x]


def build(variants):
    from ddrl_amd import build as B
    for v in variants:
        lib, bd = paths(v)
        print(B.build(extra_flags=flags(v), lib=lib, build_dir=bd), flush=True)


def run(n, variants):
    import subprocess
    for v in variants:
        lib, _ = paths(v)
        out = subprocess.run([sys.executable, __file__, "one", lib, str(n)], capture_output=True, text=True, timeout=180)
        print(f"{v or 'baseline':28s} {out.stdout.strip()} {out.stderr.strip()[-200:]}", flush=True)


def one(lib, n, env="QuantrupedMultiEnv_Local"):
    """us per sequential minibatch step of the fused update of `env` (Local: 4 policies, d = 35;
    SharedDecentral: 1 policy over 4 leg agents, d = 19) at n envs, T = 200."""
    import numpy as np, torch
    from ddrl_amd import native as N
    N.load(lib)
    from ddrl_amd.spec import make_cfg
    from ddrl_amd.trainer import glorot_ffn_flat
    T = 200
    cfg, _ = make_cfg(env, n, T)
    P = cfg.n_policies
    ctx = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    for p in range(P):
        ctx.params_set(p, glorot_ffn_flat(rng, cfg.obs_dim[p], 2))
        lay = ctx.layout[p]
        r = rng.normal(size=(T * lay["C"], lay["stride"])).astype(np.float32) * 0.5
        ctx.records_set(p, r)
    R = T * ctx.layout[0]["C"]
    nb = R // 128
    sh = [torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda() for _ in range(P)]
    pe = [torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(10)]).astype(np.int32)).cuda()
          for _ in range(P)]
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        ctx.ppo_update((1 << P) - 1, sh, pe, [0.2] * P)
        ctx.synchronize()
        best = min(best, time.perf_counter() - t0)
    import hashlib
    h = hashlib.sha256()
    for p in range(P):
        h.update(ctx.params_get(p).tobytes())
        for a in ctx.adam_get(p)[:2]:
            h.update(np.asarray(a).tobytes())
    # digest of the trained state: variants that claim bit-identical arithmetic must agree
    print(f"{best / (10 * nb) * 1e6:.2f} us/step state {h.hexdigest()[:16]}")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2:] or VARIANTS)
    elif sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 512, sys.argv[3:] or VARIANTS)
    else:
        one(sys.argv[2], int(sys.argv[3]), *sys.argv[4:5])
