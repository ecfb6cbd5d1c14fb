"""CPU check of the short-horizon parity criterion itself (tests/gpu_harness.strict_params_check,
VERDICT r2 item 7): an independent fp32 run of the same schedule (minibatch rows summed in
another order -- the kind of rounding difference the HIP kernels have) passes with no entry
beyond 1e-5 of the fp64 trajectory, and a parameter moved by 3e-5 is caught unless its fp64
gradient sits below the fp32 floor."""
import numpy as np
import pytest

from oracle import ddrl_oracle as O
from tests.gpu_harness import strict_params_check


def _case(seed, R=384):
    rng = np.random.default_rng(seed)
    d, A = 35, 2
    shapes = O.ffn_param_shapes(d, 2 * A)
    params = {k: v.astype(np.float32) for k, v in O.ffn_init(rng, d, 2 * A).items()}
    obs = rng.standard_normal((R, d)).astype(np.float32)
    lg, v, _ = O.ffn_forward(params, obs)
    act = (lg[:, :A] + np.exp(lg[:, A:]) * rng.standard_normal((R, A))).astype(np.float32)
    batch = dict(obs=obs, actions=act, logits=(lg + 0.01 * rng.standard_normal(lg.shape)).astype(np.float32),
                 logp=O.dg_logp(lg, act).astype(np.float32), vf_preds=v.astype(np.float32),
                 adv=rng.standard_normal(R).astype(np.float32), vt=(v + rng.standard_normal(R)).astype(np.float32))
    sh, pe = O.sgd_schedule(np.random.default_rng(seed + 1), R, 128, 10)
    return shapes, params, batch, sh, pe


def _reordered_run(shapes, params, batch, sh, pe, steps):
    order = np.random.default_rng(7).permutation(128)
    nb = sh.size // 128
    sh2 = sh.copy()
    sh2[:nb * 128] = sh[:nb * 128].reshape(nb, 128)[:, order].reshape(-1)
    n = sum(int(np.prod(s)) for _, s in shapes)
    new, _ = O.ppo_update("ffn", params, shapes, O.Adam(n), batch, sh2, pe, np.float32(0.2),
                          {"entropy_coeff": 0.0}, steps=steps)
    return O.pack(new, shapes)


@pytest.mark.parametrize("steps", [1, 3])
def test_reordered_fp32_run_meets_the_criterion(steps):
    shapes, params, batch, sh, pe = _case(3)
    got = _reordered_run(shapes, params, batch, sh, pe, steps)
    n_over, n_ex, n = strict_params_check(got, "ffn", params, shapes, batch, sh, pe, 0.2, steps, msg="cpu")
    assert n_over == 0 and n_ex < n


def test_a_moved_parameter_is_caught():
    shapes, params, batch, sh, pe = _case(4)
    got = _reordered_run(shapes, params, batch, sh, pe, 2).astype(np.float64)
    # fc_out/kernel's largest-gradient entries are never exemptible: move the first one
    off = sum(int(np.prod(s)) for k, s in shapes[:shapes.index(next(x for x in shapes if x[0] == "fc_out/kernel"))])
    got[off] += 3e-5
    with pytest.raises(AssertionError):
        strict_params_check(got, "ffn", params, shapes, batch, sh, pe, 0.2, 2, msg="cpu")
