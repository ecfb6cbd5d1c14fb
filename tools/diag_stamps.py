"""Per-phase cycle breakdown of the fused update kernel (diagnostic build with s_memtime
stamps; only the shares are meaningful, the stamps themselves cost a little)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from ddrl_amd import build, native as N
extra = os.environ.get("DDRL_EXTRA_FLAGS", "").split()
tag = "".join(ch for ch in "".join(extra) if ch.isalnum())[:24]
# prebuilt (here, on the CPU) when DDRL_STAMPS_LIB names it: python tools/diag_stamps.py --build
# DDRL_STAMPS_LIB=1: libddrl_hip_stamps.so; any other value: that file name in ddrl_amd/ (variants)
_sl = os.environ.get("DDRL_STAMPS_LIB", "1")
stamps_lib = os.path.join(os.path.dirname(N.LIB_PATH), "libddrl_hip_stamps.so" if _sl in ("", "1") else _sl)
if "--build" in sys.argv or not os.environ.get("DDRL_STAMPS_LIB"):
    lib = build.build(extra_flags=["-DDDRL_STAMPS"] + extra,
                      lib=stamps_lib if "--build" in sys.argv else
                      os.path.join(os.path.dirname(N.LIB_PATH), f"libddrl_hip_diag{tag}.so"),
                      build_dir=os.path.join(os.path.dirname(N.LIB_PATH), f"_build_diag{tag}"))
    if "--build" in sys.argv:
        print(lib)
        sys.exit(0)
else:
    lib = stamps_lib
N.load(lib)
from ddrl_amd.spec import make_cfg
from ddrl_amd.trainer import glorot_ffn_flat
n, T = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 512, 200
cfg, inst = make_cfg("QuantrupedMultiEnv_Local", n, T)
ctx = N.Context(cfg, 0, torch.cuda.current_stream().cuda_stream)
rng = np.random.default_rng(0)
for p in range(4):
    ctx.params_set(p, glorot_ffn_flat(rng, 35, 2))
recs = []
for p in range(4):
    lay = ctx.layout[p]
    r = rng.normal(size=(T * lay["C"], lay["stride"])).astype(np.float32) * 0.5
    r[:, lay["logit"] + 2:lay["logit"] + 4] = -0.5
    ctx.records_set(p, r)
R = T * n; nb = R // 128
sh = [torch.from_numpy(rng.permutation(R).astype(np.int32)).cuda() for _ in range(4)]
pe = [torch.from_numpy(np.stack([rng.permutation(nb) for _ in range(10)]).astype(np.int32)).cuda() for _ in range(4)]
steps = 10 * nb
for it in range(2):
    t0 = time.perf_counter()
    ctx.ppo_update(0xF, sh, pe, [0.2] * 4)
    ctx.synchronize()
    dt = time.perf_counter() - t0
st = (ctypes.c_ulonglong * (32 * 16))()
assert N.load().ddrl_diag_stamps(st) == 0
split = os.environ.get("DDRL_UPDATE_SPLIT", "2") != "1"
blocks = [0, 8, 16] if split else [0, 8]
labels = ["policy rows 0-63", "policy rows 64-127", "value rows 0-63"] if split else ["policy", "value"]
a = np.array(st, dtype=np.float64).reshape(32, 16)[blocks, :15] / steps
names = ["fwd", "loss", "dpp head/bias", "head bwd+db2+stores", "layer2 bwd+db1", "sync#1 (+gs/stats out)",
         "dW2 tiles (+out)", "sync#2", "X/dZ1 stores + sync#3", "prefetch issue", "dW1 tiles",
         "norm exchange", "adam", "sync#6", "partner exchange (split)"]
print(f"steps {steps}, {dt / steps * 1e6:.2f} us/step wall")
for wg in range(len(blocks)):
    tot = a[wg].sum()
    print(f"{labels[wg]} WG: {tot:.0f} cycles/step")
    for k, nm in enumerate(names):
        print(f"   {nm:45s} {a[wg, k]:8.0f}  {100 * a[wg, k] / tot:5.1f}%")
