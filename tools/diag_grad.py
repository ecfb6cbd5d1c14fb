"""Per-tensor gradient comparison of ddrl_ppo_grad against the oracle (diagnostic)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from oracle import ddrl_oracle as O
from tests.gpu_harness import init_params, make_ctx, run_rollout

env, n, T = "QuantrupedMultiEnv_Local", 64, 4
ctx, cfg, inst = make_ctx(env, n, T)
rng = np.random.default_rng(4)
hs = float(sys.argv[1]) if len(sys.argv) > 1 else 30.0
params = init_params(ctx, cfg, 8, head_scale=hs)
filt = (1000.0, rng.normal(size=43) * 0.3, np.abs(rng.normal(size=43)) * 999.0 + 10.0)
orc, norms, _, _ = run_rollout(ctx, cfg, inst, params, rng, filt, T)
p = 0
lay = ctx.layout[p]
rec = orc.flat_records(p, lay)
ctx.records_set(p, rec)
ctx.adv_norm_set(p, *norms[p])
rows = np.arange(128, dtype=np.int32)
g = torch.zeros(ctx.n_params[p], device="cuda")
ctx.ppo_grad(p, torch.from_numpy(rows).cuda(), 128, 0.2, g)
ctx.synchronize()
gg = g.cpu().numpy()
mean, den = norms[p]
d, A = 35, 2
sl = dict(obs=rec[rows, :d], actions=rec[rows, lay["act"]:lay["act"]+A], logits=rec[rows, lay["logit"]:lay["logit"]+2*A],
          logp=rec[rows, lay["logp"]], vf=rec[rows, lay["vf"]], adv=((rec[rows, lay["adv"]]-mean)/den).astype(np.float32), vt=rec[rows, lay["vt"]])
logits, value, cache = O.ffn_forward(params[p], sl["obs"])
print("max |logits - old logits| (should be ~0 at step 0):", np.abs(logits - sl["logits"]).max())
print("logp recompute vs stored:", np.abs(O.dg_logp(logits, sl["actions"]) - sl["logp"]).max())
dl, dv, st = O.ppo_loss_rows(logits, value, sl["actions"], sl["logits"], sl["logp"], sl["vf"], sl["adv"], sl["vt"], np.float32(0.2))
print("oracle stats", st)
shapes = O.ffn_param_shapes(d, 2*A)
gref = O.ffn_backward(params[p], cache, dl, dv)
off = 0
for name, shp in shapes:
    k = int(np.prod(shp)); a = gg[off:off+k]; b = gref[name].reshape(-1); off += k
    err = np.abs(a-b).max(); print(f"{name:22s} max|ref| {np.abs(b).max():10.4g} max err {err:10.4g} rel {err/max(1e-30,np.abs(b).max()):.3g}")
print("dlogits rows with big |d|:", np.abs(dl).max(0))
