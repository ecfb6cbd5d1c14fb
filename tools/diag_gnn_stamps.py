"""Per-phase timeline of the GNN training step (C5): the -DDDRL_GNN_STAMPS diagnostic build
stamps s_memrealtime (100 MHz, chip-wide) at the phase boundaries of the gradient launch
(thread 0 of tile 0's workgroups: actor / critic x 4 backward shares) and at the start / end of
block 0 of the reduction and Adam launches.  Prints the median over steps of each phase, in us,
relative to the earliest gradient-workgroup start of the step.

    python tools/diag_gnn_stamps.py --build          # here: prebuild libddrl_hip_gstamps.so
    python tools/diag_gnn_stamps.py [n_envs] [layer]  # GPU box
"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from ddrl_amd import build, native as N

LIB = os.path.join(os.path.dirname(N.LIB_PATH), "libddrl_hip_gstamps.so")
if "--build" in sys.argv:
    print(build.build(extra_flags=["-DDDRL_GNN_STAMPS"], lib=LIB,
                      build_dir=os.path.join(os.path.dirname(N.LIB_PATH), "_build_gstamps")))
    sys.exit(0)

import torch

N.load(LIB)
from ddrl_amd.models import glorot_gnn_flat
from ddrl_amd.spec import make_cfg
from ddrl_amd.synthetic import SyntheticRollout

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 2048
layer = args[1] if len(args) > 1 else "mpnn"
T, STEPS, SKIP = 200, 4000, 500
cfg, _ = make_cfg("QuantrupedMultiEnv_DecentralShared_Graph", n, T,
                  {"model": {"custom_model": "gnn", "gnn_layer": layer}})
ctx = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
ctx.params_set(0, glorot_gnn_flat(np.random.default_rng(0), cfg.act_dim, layer=layer))
syn = SyntheticRollout(n, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=0)
ctx.observe(syn.obs[0])
ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, syn.dones_for_fragment(), syn.actions)
ctx.gae()
R = T * ctx.layout[0]["C"]
nb = R // 128
rng = np.random.default_rng(1)
sh = torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda()
pe = torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(10)]).astype(np.int32)).cuda()
ctx.ppo_update(1, [sh], [pe], [0.2], max_steps=200)   # warm
ctx.synchronize()
t0 = time.perf_counter()
ctx.ppo_update(1, [sh], [pe], [0.2], max_steps=STEPS)
ctx.synchronize()
wall = (time.perf_counter() - t0) / STEPS * 1e6
buf = (ctypes.c_ulonglong * (4096 * 9 * 12))()
span = (ctypes.c_ulonglong * (4096 * 3 * 256 * 2))()
assert N.load().ddrl_diag_gnn_stamps(buf, span) == 0
a = np.array(buf, dtype=np.float64).reshape(4096, 9, 12)[SKIP:STEPS]
sp = np.array(span, dtype=np.float64).reshape(4096, 3, 256, 2)[SKIP:STEPS]
g = a[:, :8, :]                      # gradient workgroups [step][wg][k]
t_start = sp[:, 0, :, 0].min(1)      # earliest gradient-WG start of the step (any tile)
rel = lambda x: (x - t_start[:, None]) * 0.01 if x.ndim == 2 else (x - t_start) * 0.01   # ticks -> us
names = ["start", "hypernet MFMA/tanh + sync", "h finalize + sync", "message passing", "head + loss + sync",
         "dWout / du / layer bwd (dh)", "layer dW tiles", "sync (dz)", "qt + sync", "hypernet bwd (end)"]
print(f"C5 n_envs={n} layer={layer}: {wall:.2f} us/step wall over {STEPS} steps (diagnostic build)")
print("gradient workgroups of tile 0, median us from the step's first WG start (actor z0..3 | critic z0..3):")
for k, nm in [(0, names[0]), (10, "weights / records landed")] + list(enumerate(names))[1:]:
    vals = np.median(rel(g[:, :, k]), axis=0)
    print(f"  {k:2d} {nm:30s} " + " ".join(f"{v:6.2f}" for v in vals))
print("every workgroup of the three launches (median over steps, us from the step's first gradient WG start):")
for L, nm in enumerate(["gradient", "reduction", "adam"]):
    st, en = sp[:, L, :, 0], sp[:, L, :, 1]
    used = (st > 0).all(0) & (en > 0).all(0)
    st, en = st[:, used], en[:, used]
    print(f"  {nm:10s} ({used.sum():3d} WGs): first start {np.median((st.min(1) - t_start) * 0.01):6.2f}  "
          f"last start {np.median((st.max(1) - t_start) * 0.01):6.2f}  first end {np.median((en.min(1) - t_start) * 0.01):6.2f}  "
          f"last end {np.median((en.max(1) - t_start) * 0.01):6.2f}")
r = a[:, 8, :]
grad_end = g[:, :, 9].max(1)
print("reduction / Adam (block 0), median us from the step's first WG start:")
for k, nm in enumerate(["reduce start", "reduce block0 end", "adam start", "adam block0 end"]):
    print(f"  {nm:20s} {np.median(rel(r[:, k])):6.2f}")
nxt = t_start[1:] - r[:-1, 3]
print(f"  gap last tile-0 WG end -> reduce start {np.median((r[:, 0] - grad_end) * 0.01):6.2f} us")
print(f"  gap adam block0 end -> next step's first gradient WG start {np.median(nxt * 0.01):6.2f} us")
print(f"  step period (first WG start to next) {np.median(np.diff(t_start)) * 0.01:6.2f} us")
