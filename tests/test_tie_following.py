"""CPU checks of the tie-following parity machinery itself (tests/gpu_harness.
tie_following_trajectory, DESIGN.md section 4 "Near-ties"), without a GPU:

* the numpy fp32 walk (NumpyLockstep), one step at a time, is oracle.ppo_update bit for bit --
  its distance from the fp64 trajectory that follows it is the e32(H) of the Local bar;
* an "implementation" that is the fp64 algorithm itself except for clip decisions it takes the
  other way at chosen steps (the smallest-margin decision of that step's minibatch, as a rounding
  difference would pick) is found exactly: the helper reports those steps, kinds and rows and
  nothing else, and the trajectory it returns is the implementation's bit for bit, while the
  plain fp64 trajectory has left it.
"""
import numpy as np

from oracle import ddrl_oracle as O
from tests.gpu_harness import NumpyLockstep, tie_following_trajectory

O64 = O.with_dtype(np.float64)


def _case(seed=3, R=128 * 12):
    rng = np.random.default_rng(seed)
    d, A = 35, 2
    shapes = O.ffn_param_shapes(d, 2 * A)
    params = {k: v.astype(np.float32) for k, v in O.ffn_init(rng, d, 2 * A).items()}
    obs = rng.standard_normal((R, d)).astype(np.float32)
    lg, v, _ = O.ffn_forward(params, obs)
    act = (lg[:, :A] + np.exp(lg[:, A:]) * rng.standard_normal((R, A))).astype(np.float32)
    # a sixth of the rows near the value clip: |V - vf_old| within 0.2 % of vf_clip = 10
    near = rng.random(R) < 1 / 6
    vf_old = np.where(near, v + np.sign(rng.standard_normal(R)) * 10 * (1 + 2e-3 * rng.uniform(-1, 1, R)), v)
    batch = dict(obs=obs, actions=act, logits=(lg + 0.01 * rng.standard_normal(lg.shape)).astype(np.float32),
                 logp=O.dg_logp(lg, act).astype(np.float32), vf_preds=vf_old.astype(np.float32),
                 adv=rng.standard_normal(R).astype(np.float32),
                 vt=(v + 8.0 * rng.standard_normal(R)).astype(np.float32))
    sh, pe = O.sgd_schedule(np.random.default_rng(seed + 1), R, 128, 10)
    return shapes, params, batch, sh, pe


class _FlippingFp64:
    """The fp64 minibatch loop, except that at each step k of `flip_steps` ({k: "pol" | "vf"}) the
    decision of that kind with the smallest margin in the minibatch is taken the other way."""

    def __init__(self, params, shapes, batch, sh, pe, kl, flip_steps):
        self.shapes, self.batch, self.sh, self.pe, self.kl = shapes, batch, sh, pe, kl
        self.th = O64.pack({k: v.astype(np.float64) for k, v in params.items()}, shapes)
        self.adam = O64.Adam(self.th.size)
        self.flip_steps, self.flipped, self.snaps, self.k = dict(flip_steps), [], {}, 0

    def _grads(self, rows, record):
        b, p = self.batch, O64.unpack(self.th, self.shapes)
        logits, value, cache = O64.ffn_forward(p, b["obs"][rows])
        args = [b[c][rows] for c in ("actions", "logits", "logp", "vf_preds", "adv", "vt")]
        force = None
        if self.k in self.flip_steps:
            pol_on, pol_m, vf_on, m_sq, m_in = O.ppo_branches(logits, value, args[0], args[2], args[3], args[4],
                                                              args[5])
            vm = np.where(m_in > 0, m_in, np.minimum(np.abs(m_in), np.abs(m_sq)))
            kind = self.flip_steps[self.k]
            if kind == "pol":
                cand = min((abs(float(pol_m[i])), "pol", i, bool(pol_on[i])) for i in range(rows.size))
            else:
                cand = min((abs(float(vm[i])), "vf", i, bool(vf_on[i])) for i in range(rows.size))
            force = {"pol": {}, "vf": {}}
            force[cand[1]][cand[2]] = not cand[3]
            if record:
                self.flipped.append((self.k, cand[1], cand[2]))
        dl, dv, _ = O64.ppo_loss_rows(logits, value, *args, np.float64(self.kl), force=force)
        g = O64.ffn_backward(p, cache, dl, dv)
        return [g[nm] for nm, _ in self.shapes]

    def grad(self, rows):
        return np.concatenate([g.reshape(-1) for g in self._grads(rows, False)])

    def step(self, k):
        assert k == self.k
        nb = self.pe.shape[1]
        rows = O.minibatch_rows(self.sh, self.pe, k // nb, k % nb)
        clipped, _ = O64.clip_by_global_norm(self._grads(rows, True))
        self.th = self.adam.apply(self.th, np.concatenate([c.reshape(-1) for c in clipped]))
        self.k += 1

    def theta(self):
        return self.th.copy()


def test_numpy_lockstep_is_ppo_update_bit_for_bit():
    shapes, params, batch, sh, pe = _case()
    horizons = [1, 7, 40, 120]
    npl = NumpyLockstep(params, shapes, batch, sh, pe, 0.2)
    tf, _, ties = tie_following_trajectory(None, 0, params, shapes, batch, sh, pe, 0.2, max(horizons), horizons,
                                           impl=npl)
    snaps = {h: None for h in horizons}
    n = O.pack(params, shapes).size
    O.ppo_update("ffn", params, shapes, O.Adam(n), batch, sh, pe, 0.2, {}, steps=max(horizons), snapshots=snaps)
    for h in horizons:
        assert np.array_equal(npl.snaps[h], snaps[h].astype(np.float64)), h
        assert np.abs(npl.snaps[h] - tf[h]).max() < 1e-5, h      # fp32 drift only, at these horizons


def test_flipped_decisions_are_found_and_followed_exactly():
    shapes, params, batch, sh, pe = _case()
    horizons = [10, 60, 120]
    impl = _FlippingFp64(params, shapes, batch, sh, pe, 0.2, flip_steps={5: "pol", 33: "vf", 77: "vf", 101: "pol"})
    missed = []
    tf, stats, ties = tie_following_trajectory(None, 0, params, shapes, batch, sh, pe, 0.2, max(horizons), horizons,
                                               impl=impl, missed=missed)
    assert not missed
    assert [(t[0], t[1], t[2]) for t in ties] == impl.flipped
    assert {t[1] for t in ties} == {"pol", "vf"}
    assert all(t[6] <= 1e-12 and t[7] > 1e-4 for t in ties), ties   # explained exactly; fp64's outcome is not
    assert len(stats) == max(horizons)
    plain = {h: None for h in horizons}
    n = O.pack(params, shapes).size
    O64.ppo_update("ffn", {k: v.astype(np.float64) for k, v in params.items()}, shapes, O64.Adam(n), batch, sh, pe,
                   0.2, {}, steps=max(horizons), snapshots=plain)
    for h in horizons:
        assert np.array_equal(tf[h], impl.snaps[h]), h
        assert np.abs(np.asarray(plain[h]) - impl.snaps[h]).max() > 1e-6, h   # the flips matter


def test_a_flip_outside_the_candidate_pool_is_reported():
    """With a pool too small to hold the flipped decision (the value rows near the clip have the
    smaller margins), the step is reported as unexplained rather than silently passed over."""
    shapes, params, batch, sh, pe = _case()
    impl = _FlippingFp64(params, shapes, batch, sh, pe, 0.2, flip_steps={5: "pol"})
    missed = []
    tie_following_trajectory(None, 0, params, shapes, batch, sh, pe, 0.2, 8, [8], impl=impl, pool=4, missed=missed)
    assert missed and missed[0][0] == 5, missed
