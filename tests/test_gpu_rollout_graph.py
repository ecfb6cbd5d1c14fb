"""ddrl_rollout_fragment as a captured HIP graph vs the same launches issued one by one.

The library captures the fragment's T x (act, reward, filter push, observe) + bootstrap
launches into one graph on first use and re-launches it while the call's buffers are the same
(every other kernel argument is fixed at context creation).  Two contexts of the same data --
DDRL_ROLLOUT_GRAPH=0 (direct launches) and the default -- run three fragments each; the buffers'
contents change between fragments (new synthetic draws written in place), the second and third
re-use the graph, and a fourth call with a different done buffer re-captures.  Records, last
values, the env-side filter state and the standardization sums must be bit-identical.  (The
rollout kernels themselves are checked against the oracle in tests/test_gpu_parity.py and
tests/test_gpu_fullsize.py, which run through the graph.)
"""
import os

import numpy as np
import pytest

from tests.gpu_harness import init_params, make_ctx

pytestmark = pytest.mark.gpu
ENV, N, T = "QuantrupedMultiEnv_Local", 96, 12


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _ctx(**envvars):
    old = {k: os.environ.get(k) for k in envvars}
    os.environ.update({k: str(v) for k, v in envvars.items()})
    try:
        return make_ctx(ENV, N, T)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _run(**envvars):
    import torch
    from ddrl_amd.synthetic import SyntheticRollout
    ctx, cfg, _ = _ctx(**envvars)
    init_params(ctx, cfg, 3, head_scale=1.0)
    syn = SyntheticRollout(N, T, cfg.obs_full_dim, cfg.n_agents, cfg.act_dim, "cuda:0", seed=9)
    gen = torch.Generator(device="cuda:0")
    gen.manual_seed(17)
    ctx.observe(syn.obs[0])
    out = []
    for k in range(4):
        done = syn.dones_for_fragment()
        if k == 3:
            done = done.clone()   # another buffer: a new capture
        ctx.rollout_fragment(syn.obs, syn.eps, syn.fw, syn.cfrc, done, syn.actions)
        ctx.gae()
        ctx.synchronize()
        out.append([ctx.records_get(p).copy() for p in range(cfg.n_policies)] +
                   [ctx.last_values_get(p).copy() for p in range(cfg.n_policies)] +
                   [np.asarray(x).copy() for x in ctx.filter_get()] +
                   [np.asarray(ctx.adv_sums_get(p)).copy() for p in range(cfg.n_policies)])
        for buf in (syn.obs, syn.eps, syn.fw, syn.cfrc):   # new contents, same addresses
            buf.copy_(torch.randn(buf.shape, device="cuda:0", generator=gen))
    ctx.close()
    return out


def test_rollout_graph_matches_direct_launches_bit_for_bit():
    direct = _run(DDRL_ROLLOUT_GRAPH=0)
    graph = _run()
    assert len(direct) == len(graph) == 4
    for a, b in zip(direct, graph):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    # the fragments differ from each other (the graph really re-read the buffers)
    assert not np.array_equal(graph[0][0], graph[1][0])
