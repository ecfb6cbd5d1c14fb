"""The published QuantrupedMultiEnv_Local policies (checkpoint 1250, 20M env steps; fixture
tests/golden/ckpt_local_1250.npz from the no-code reader) through the HIP path against the
oracle: weights, Adam m / v, beta powers and the RLlib per-policy
MeanStdFilter (observation_filter = MeanStdFilter, as the published runs trained) go in
through ddrl_params_set / ddrl_adam_set / ddrl_policy_filter_set; a rollout with GAE, then
three fused update steps, are compared with the oracle started from the same state.
Tolerances as tests/test_gpu_parity.py (outputs 1e-5 relative + 2e-5 absolute; parameters
>= 99.9 % within 1e-5, max <= 2 lr steps)."""
import json
import os

import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import make_ctx, run_rollout, strict_params_check

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ckpt_local_1250.npz")


def _close(a, b, rtol=1e-5, atol=2e-5, msg=""):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=msg)


def test_published_local_policies_rollout_and_update():
    import torch
    z = np.load(FIX, allow_pickle=False)
    pids = json.loads(bytes(z["policy_ids"]).decode())
    n, T = 40, 8
    ctx, cfg, inst = make_ctx("QuantrupedMultiEnv_Local", n, T, {"observation_filter": "MeanStdFilter"})
    assert cfg.policy_filter == 1
    names = list(type(inst).policy_names)
    shapes = O.ffn_param_shapes(35, 4)
    params, pfilt, adams = [], [], []
    for p, name in enumerate(names):
        assert name in pids
        w = z[f"{name}/weights"]
        ctx.params_set(p, w)
        b1p, b2p = (float(x) for x in z[f"{name}/beta_powers"])
        ctx.adam_set(p, z[f"{name}/adam_m"], z[f"{name}/adam_v"], b1p, b2p)
        params.append(O.unpack(w, shapes))
        pfilt.append((float(z[f"{name}/filter_n"][0]), z[f"{name}/filter_M"], z[f"{name}/filter_S"]))
        a = O.Adam(w.size, lr=cfg.lr)
        a.m, a.v = z[f"{name}/adam_m"].copy(), z[f"{name}/adam_v"].copy()
        a.b1p, a.b2p = np.float32(b1p), np.float32(b2p)
        adams.append(a)
    import copy
    adam0 = copy.deepcopy(adams)      # the published optimizer state, before the oracle steps it
    np.testing.assert_array_equal(ctx.params_get(0), z[f"{names[0]}/weights"])   # round trip
    rng = np.random.default_rng(23)
    filt = (1000.0, rng.normal(size=43) * 0.3, np.abs(rng.normal(size=43)) * 999.0 + 10.0)
    orc, norms, a_gpu, a_orc = run_rollout(ctx, cfg, inst, params, rng, filt, T, pfilt=pfilt)
    _close(a_gpu, a_orc, msg="env actions")
    for p in range(4):
        lay = ctx.layout[p]
        got, ref = ctx.records_get(p), orc.flat_records(p, lay)
        for name, sl in [("obs", slice(0, 35)), ("logits", slice(lay["logit"], lay["logit"] + 4)),
                         ("logp", lay["logp"]), ("vf", lay["vf"]), ("adv", lay["adv"]), ("vt", lay["vt"])]:
            _close(got[:, sl], ref[:, sl], msg=f"p{p} {name}")
        pn, pM, pS = ctx.policy_filter_get(p)
        assert pn == orc.pf[p].n
        _close(pM, orc.pf[p].M, rtol=1e-10, atol=1e-10)
    # three fused steps from the published optimizer state, on the oracle's batch
    steps, kls = 3, [float(z[f"{nm}/kl_coeff"][0]) for nm in names]
    sh_l, pe_l = [], []
    for p in range(4):
        lay = ctx.layout[p]
        ctx.records_set(p, orc.flat_records(p, lay))
        ctx.adv_norm_set(p, *norms[p])
        sh, pe = O.sgd_schedule(np.random.default_rng(60 + p), T * lay["C"], 128, cfg.num_sgd_iter)
        sh_l.append(sh)
        pe_l.append(pe)
    ctx.ppo_update(0xF, [torch.from_numpy(s).cuda() for s in sh_l], [torch.from_numpy(s).cuda() for s in pe_l],
                   kls, max_steps=steps)
    ctx.synchronize()
    for p in range(4):
        lay = ctx.layout[p]
        rec = orc.flat_records(p, lay)
        mean, den = norms[p]
        batch = dict(obs=rec[:, :35], actions=rec[:, lay["act"]:lay["act"] + 2],
                     logits=rec[:, lay["logit"]:lay["logit"] + 4], logp=rec[:, lay["logp"]],
                     vf_preds=rec[:, lay["vf"]], adv=((rec[:, lay["adv"]] - mean) / den).astype(np.float32),
                     vt=rec[:, lay["vt"]])
        new, _ = O.ppo_update("ffn", params[p], shapes, adams[p], batch, sh_l[p], pe_l[p], np.float32(kls[p]),
                              {"entropy_coeff": 0.0}, steps=steps)
        want = O.pack(new, shapes)
        diff = np.abs(ctx.params_get(p) - want)
        assert np.mean(diff <= 1e-5 + 1e-5 * np.abs(want)) >= 0.999, diff.max()
        assert diff.max() <= 2 * cfg.lr * steps + 1e-5
        strict_params_check(ctx.params_get(p), "ffn", params[p], shapes, batch, sh_l[p], pe_l[p], kls[p], steps,
                            adam=adam0[p], lr=float(adam0[p].lr), msg=f"published {names[p]}")
        m, v, b1p, b2p = ctx.adam_get(p)
        _close(m, adams[p].m, rtol=1e-4, atol=1e-7, msg="Adam m")
        assert b1p == np.float32(adams[p].b1p) and b2p == np.float32(adams[p].b2p)
    ctx.close()
