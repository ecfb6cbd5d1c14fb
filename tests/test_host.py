"""Host-side mirror of the reference's plugin surface (no GPU): env registry, policy
mapping, spaces, and the routing tables `make_cfg` hands to the kernels.

Reference: simulation_envs/__init__.py:53-67 (registry), the env classes' return_policies /
policy_mapping_fn, and SURVEY 8(a) a1/a7/a8 for the tables (pinned separately against
tests/golden/layout_tables.json in test_oracle.py).
"""
import numpy as np
import pytest

from ddrl_amd import native as N
from ddrl_amd.simulation_envs import ENV_REGISTRY, get_env_class
from ddrl_amd.spec import make_cfg

REFERENCE_NAMES = [
    "QuantrupedMultiEnv_Centralized", "QuantrupedMultiEnv_Decentral_Graph",
    "QuantrupedMultiEnv_DecentralShared_Graph", "QuantrupedMultiEnv_FullyDecentral",
    "QuantrupedMultiEnv_FullyDecentralGlobalCost", "QuantrupedMultiEnv_SingleNeighbor",
    "QuantrupedMultiEnv_SingleDiagonal", "QuantrupedMultiEnv_SingleToFront", "QuantrupedMultiEnv_Local",
    "QuantrupedMultiEnv_TwoSides", "QuantrupedMultiEnv_TwoDiags", "QuantrupedMultiEnv_SharedDecentral",
    "QuantrupedMultiEnv_SharedDecentralLegID", "QuantrupedMultiEnv_SharedDecentralLegTransforms",
]


def test_registry_has_every_reference_multiagent_env():
    for name in REFERENCE_NAMES:
        assert name in ENV_REGISTRY, name


@pytest.mark.parametrize("name", [n for n in REFERENCE_NAMES if n != "QuantrupedMultiEnv_Decentral_Graph"])
def test_make_cfg_tables_are_consistent(name):
    cfg, inst = make_cfg(name, 8, 4)
    cls = get_env_class(name)
    pols = cls.return_policies()
    assert list(pols) == list(cls.policy_names)
    assert cfg.n_agents == len(inst.agent_names) and cfg.n_policies == len(cls.policy_names)
    for j, a in enumerate(inst.agent_names):
        p = cfg.agent_policy[j]
        assert cls.policy_names[p] == cls.policy_mapping_fn(a)
        d = cfg.obs_dim[p]
        idx = [cfg.obs_index[j][f] for f in range(d)]
        assert all(-2 <= i < cfg.obs_full_dim for i in idx)
        acts = [cfg.act_index[j][k] for k in range(cfg.act_dim)]
        assert acts == list(inst.action_indices[a])
    # every env action is driven by exactly one agent
    driven = sorted(cfg.act_index[j][k] for j in range(cfg.n_agents) for k in range(cfg.act_dim))
    assert driven == list(range(8))


def test_legid_one_hot_columns():
    cfg, inst = make_cfg("QuantrupedMultiEnv_SharedDecentralLegID", 4, 2)
    assert cfg.n_policies == 1 and cfg.obs_dim[0] == 23
    for j in range(4):
        one_hot = [cfg.obs_index[j][k] for k in range(4)]
        assert one_hot == [-2 if k == j else -1 for k in range(4)]
        assert [cfg.obs_index[j][4 + f] for f in range(19)] == list(inst.obs_indices[inst.agent_names[j]])


def test_legtransforms_negates_the_rear_right_and_front_right_knees():
    cfg, inst = make_cfg("QuantrupedMultiEnv_SharedDecentralLegTransforms", 4, 2)
    negated = sorted(cfg.act_index[j][k] for j in range(4) for k in range(2) if cfg.act_negate[j][k])
    from ddrl_amd.simulation_envs.layouts import ACTION_FIELDS
    assert [ACTION_FIELDS[i] for i in negated] == ["fr_knee", "hr_knee"]


def test_decentral_graph_has_no_consistent_model():
    with pytest.raises(ValueError, match="Appendix B.8"):
        make_cfg("QuantrupedMultiEnv_Decentral_Graph", 4, 2)


def test_graph_env_spaces_and_model_kind():
    cfg, inst = make_cfg("QuantrupedMultiEnv_DecentralShared_Graph", 4, 2)
    assert cfg.model_kind == N.MODEL_GNN and cfg.n_policies == 1 and cfg.obs_dim[0] == 19
    assert [cfg.leg_angle_deg[j] for j in range(4)] == [45.0, 135.0, -135.0, -45.0]
    adj = np.array(inst.create_adj())
    assert (adj == adj.T).all() and adj.sum() == 8 and np.trace(adj) == 0


def test_trainer_config_keys_and_update_kl():
    from ddrl_amd.trainer import update_kl
    assert update_kl(0.2, 0.03) == pytest.approx(0.3)
    assert update_kl(0.2, 0.001) == pytest.approx(0.1)
    assert update_kl(0.2, 0.01) == 0.2
    cfg, _ = make_cfg("QuantrupedMultiEnv_Local", 4, 2, {"lr": 1e-4, "num_sgd_iter": 3})
    assert cfg.lr == pytest.approx(1e-4) and cfg.num_sgd_iter == 3 and cfg.sgd_minibatch_size == 128


def test_cup_model_reads_leg_features_and_sets_coupling():
    """"cup" (models/coupling_net_glorot_uniform_init.py:32-137) on the LegID env: the model
    input is the 19 features of the (leg index, features) tuple, the leg index selects the
    coupling row; on an env without that tuple the reference model cannot be built."""
    from ddrl_amd.models import ModelCatalog
    from ddrl_amd.trainer import leg_coupling_init
    cfg, inst = make_cfg("QuantrupedMultiEnv_SharedDecentralLegID", 4, 2, {"model": {"custom_model": "cup"}})
    assert cfg.leg_coupling == 1 and cfg.obs_dim[0] == 19 and cfg.n_policies == 1
    for j, a in enumerate(inst.agent_names):
        assert list(cfg.obs_index[j][:19]) == list(inst.obs_indices[a])
    np.testing.assert_array_equal(leg_coupling_init(2).reshape(4, 2), [[1, 1], [-1, -1], [-1, -1], [1, 1]])
    assert ModelCatalog.get("cup").__name__ == "FullyConnectedNetwork_Coupling_GlorotUniformInitializer"
    with pytest.raises(ValueError):
        make_cfg("QuantrupedMultiEnv_SharedDecentral", 4, 2, {"model": {"custom_model": "cup"}})


# a5: GlorotUniformScaled (models/glorot_uniform_scaled_initializer.py:3-19) -- the product's
# host init against the oracle's ffn_init / gnn_init: same draws in the same variable order
# (bit-identical for one seed), limits sqrt(6 s / (fan_in + fan_out)) with s = 1 for hidden
# kernels and 0.01 for the output heads, zero biases.
@pytest.mark.parametrize("d,A", [(19, 2), (27, 2), (35, 2), (43, 8), (36, 2), (28, 4)])
def test_glorot_ffn_init_matches_oracle(d, A):
    from oracle import ddrl_oracle as O
    from ddrl_amd.trainer import glorot_ffn_flat
    shapes = O.ffn_param_shapes(d, 2 * A)
    ref = O.pack(O.ffn_init(np.random.default_rng(5), d, 2 * A), shapes)
    got = glorot_ffn_flat(np.random.default_rng(5), d, A)
    assert got.dtype == np.float32 and got.shape == ref.shape
    np.testing.assert_array_equal(got, ref)
    parts = O.unpack(got, shapes)
    for name, shape in shapes:
        w = parts[name]
        if name.endswith("bias"):
            assert not w.any(), name
            continue
        s = 0.01 if name.startswith(("fc_out", "value_out")) else 1.0
        lim = np.sqrt(6.0 * s / (shape[0] + shape[1]))
        assert np.abs(w).max() <= lim and np.abs(w).max() > 0.9 * lim, name


@pytest.mark.parametrize("A", [2, 4])
def test_glorot_gnn_init_matches_oracle(A):
    from oracle import ddrl_oracle as O
    from ddrl_amd.models import glorot_gnn_flat
    shapes = O.gnn_param_shapes(2 * A)
    ref = O.pack(O.gnn_init(np.random.default_rng(6), 2 * A), shapes)
    got = glorot_gnn_flat(np.random.default_rng(6), A)
    np.testing.assert_array_equal(got, ref)
    parts = O.unpack(got, shapes)
    for name, shape in shapes:
        w = parts[name]
        if name.endswith("bias"):
            assert not w.any(), name
            continue
        s = 0.01 if "linear_out" in name else 1.0
        lim = np.sqrt(6.0 * s / (shape[0] + shape[1]))
        assert np.abs(w).max() <= lim and np.abs(w).max() > 0.9 * lim, name


def test_rank_seeds_differ_per_rank_and_keep_rank0():
    from ddrl_amd.trainer import rank_seeds
    seeds = [rank_seeds(3, r) for r in range(8)]
    assert seeds[0] == (3, 4)                     # single-process seeds unchanged
    flat = [s for pair in seeds for s in pair]
    assert len(set(flat)) == len(flat)            # no two ranks (or streams) share a seed
