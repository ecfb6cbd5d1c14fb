"""Ablation timing of the GNN minibatch step (variants skip a phase; timing only).

    python tools/ablate_gnn.py build      # container
    python tools/ablate_gnn.py run        # GPU box
"""
import os, subprocess, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
VARIANTS = ["", "DDRL_ABL_GNN_NO_HBWD", "DDRL_ABL_GNN_NO_HFWD", "DDRL_ABL_GNN_EMPTY", "DDRL_ABL_GNN_GRAD_ONLY",
            "DDRL_ABL_GNN_EMPTY -DDDRL_ABL_GNN_GRAD_ONLY"]


def paths(v):
    from ddrl_amd import native as N
    d = os.path.dirname(N.LIB_PATH)
    tag = v.replace("DDRL_ABL_GNN_", "").replace(" -D", "_").lower() or "base"
    return os.path.join(d, f"libddrl_hip_gabl_{tag}.so"), os.path.join(d, f"_build_gabl_{tag}")


def one(lib):
    import numpy as np, torch
    from ddrl_amd import native as N
    N.load(lib)
    from ddrl_amd.spec import make_cfg
    from ddrl_amd.models import glorot_gnn_flat
    n, T = 128, 200
    cfg, _ = make_cfg("QuantrupedMultiEnv_DecentralShared_Graph", n, T)
    ctx = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
    rng = np.random.default_rng(0)
    ctx.params_set(0, glorot_gnn_flat(rng, 2))
    lay = ctx.layout[0]
    R = T * lay["C"]
    r = rng.normal(size=(R, lay["stride"])).astype(np.float32) * 0.5
    r[:, 92] = np.tile(np.arange(4), R // 4)
    ctx.records_set(0, r)
    nb = R // 128
    sh = torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda()
    pe = torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(10)]).astype(np.int32)).cuda()
    steps = 2000
    ctx.ppo_update(1, [sh], [pe], [0.2], max_steps=100)
    ctx.synchronize()
    t0 = time.perf_counter()
    ctx.ppo_update(1, [sh], [pe], [0.2], max_steps=steps)
    t1 = time.perf_counter()
    ctx.synchronize()
    t2 = time.perf_counter()
    print(f"{(t2 - t0) / steps * 1e6:.2f} us/step (host enqueue {(t1 - t0) / steps * 1e6:.2f} us/step)")


if __name__ == "__main__":
    if sys.argv[1] == "build":
        from ddrl_amd import build as B
        for v in VARIANTS:
            lib, bd = paths(v)
            print(B.build(extra_flags=[f"-D{v}"] if v else [], lib=lib, build_dir=bd), flush=True)
    elif sys.argv[1] == "run":
        for v in VARIANTS:
            out = subprocess.run([sys.executable, __file__, "one", paths(v)[0]], capture_output=True, text=True)
            print(f"{v or 'baseline':26s} {out.stdout.strip()} {out.stderr.strip()[-160:]}", flush=True)
    else:
        one(sys.argv[2])
