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


# f1: the host env plane's stand-in envs (hostenv.cpp) -- deterministic, thread-count
# invariant, the reference env's observation layout (no GPU needed: unpinned buffers here)
def test_host_env_plane_is_deterministic_and_thread_invariant():
    runs = []
    for threads in (1, 3):
        e = N.HostEnv(37, 44, threads, seed=5, target_velocity=0.5)
        e.reset()
        rng = np.random.default_rng(2)
        out = []
        for _ in range(60):
            e.act[:] = rng.uniform(-1.5, 1.5, size=(37, 8)).astype(np.float32)
            e.step(0, 20)
            e.step(20, 37)
            out.append((e.obs.copy(), e.fw.copy(), e.cfrc.copy(), e.done.copy()))
        runs.append(out)
        assert e.threads == threads
        e.close()
    for a, b in zip(*runs):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    obs = np.stack([o[0] for o in runs[0]])
    assert np.isfinite(obs).all()
    assert np.all(obs[:, :, 43] == np.float32(0.5))            # TVel column
    # ctrl columns 35..42 are the clipped actions of the step (0 right after a reset)
    assert np.abs(obs[:, :, 35:43]).max() <= 1.0
    quat = obs[:, :, 1:5].astype(np.float64)
    np.testing.assert_allclose(np.linalg.norm(quat, axis=-1), 1.0, atol=1e-6)
    cf = np.stack([o[2] for o in runs[0]])
    assert (cf[:, :, 0] == 0).all() and cf[:, :, 4::3, 5].max() > 0      # floor body: no force; feet touch


def test_host_env_tvel_forward_reward_matches_oracle():
    """f4: the TVel envs' forward reward (quantruped_v3.py:391-392) -- the same dynamics as the
    plain env (the target velocity is only observed), fw = the target-velocity reward of the
    torso's x velocity; 1.0 at the target, the reward of the plain env elsewhere."""
    from oracle import ddrl_oracle as O
    envs = [N.HostEnv(16, 43, 2, seed=9), N.HostEnv(16, 44, 2, seed=9, target_velocity=0.75)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(4)
    for _ in range(40):
        a = rng.uniform(-1, 1, size=(16, 8)).astype(np.float32)
        for e in envs:
            e.act[:] = a
            e.step()
        np.testing.assert_array_equal(envs[0].obs, envs[1].obs[:, :43])
        np.testing.assert_allclose(envs[1].fw, O.tvel_forward_reward(envs[0].fw.astype(np.float64), 0.75),
                                   rtol=1e-5, atol=1e-6)
    assert O.tvel_forward_reward(0.75, 0.75) == pytest.approx(1.0)
    for e in envs:
        e.close()


def test_host_env_rejects_bad_arguments():
    with pytest.raises(N.DdrlError):
        N.HostEnv(44 - 44, 43)
    with pytest.raises(N.DdrlError):
        N.HostEnv(8, 44)            # TVel needs a target velocity
    with pytest.raises(N.DdrlError):
        N.HostEnv(8, 40)
    e = N.HostEnv(8, 43)
    with pytest.raises(N.DdrlError):
        e.step(4, 4)
    e.close()


@pytest.mark.parametrize("env_name,config", [
    ("QuantrupedMultiEnv_Local", {}),
    ("QuantrupedMultiEnv_FullyDecentralGlobalCost", {}),
    ("QuantrupedMultiEnv_TwoSides", {"norm_reward": True}),
    ("QuantrupedMultiEnv_SharedDecentralLegTransforms", {}),
    ("QuantrupedMultiEnv_Centralized", {"target_velocity": [0.5]}),
])
def test_dict_api_over_host_env_plane_matches_oracle(env_name, config):
    """MultiAgentEnv reset() / step(action_dict) over the host env plane (ddrl_amd.hostenv):
    filter, distribute_observations, concatenate_actions and the rewards against the oracle
    on the env plane's own raw outputs (adaptor :83-85, :124-136, :160-212, :214-250)."""
    from oracle import ddrl_oracle as O
    from ddrl_amd.hostenv import HostMultiAgentEnv
    env = HostMultiAgentEnv(env_name, config, n_envs=1, seed=4)
    spec = env.spec
    rs = O.RunningStat((env.D,))
    obs = env.reset()
    ref = O.distribute_observations(O.mean_std_filter(env.env.obs[0], rs, True, 10.0), spec.obs_indices)
    assert set(obs) == set(spec.agent_names)
    for a in obs:
        np.testing.assert_allclose(obs[a], ref[a], rtol=1e-12, atol=1e-12)
    rng = np.random.default_rng(0)
    tables = {a: spec.contact_force_indices[a] for a in spec.agent_names}
    for _ in range(30):
        actions = {a: rng.uniform(-1.2, 1.2, size=len(spec.action_indices[a])) for a in spec.agent_names}
        obs, rew, done, info = env.step(actions)
        applied = env.env.act[0].astype(np.float64)
        sign = {a: np.where(np.asarray(getattr(spec, "action_negate", {}).get(a, [False] * 8))[:len(spec.action_indices[a])], -1.0, 1.0)
                for a in spec.agent_names}
        want = O.concatenate_actions({a: np.clip(v, -1, 1) * sign[a] for a, v in actions.items()}, spec.action_indices)
        np.testing.assert_allclose(applied, want.astype(np.float32))
        per_agent = {a: applied[spec.action_indices[a]] for a in spec.agent_names}
        fw, cfrc = float(env.env.fw[0]), env.env.cfrc[0].astype(np.float64)
        if spec.reward_mode == "global":
            rref = O.global_reward(fw, cfrc, per_agent, spec.ctrl_cost_weight, spec.contact_cost_weight)
        else:
            rref = O.per_leg_reward(fw, cfrc, per_agent, tables, spec.ctrl_cost_weight, spec.contact_cost_weight,
                                    norm_reward=spec.reward_mode == "norm")
        for a in spec.agent_names:
            assert rew[a] == pytest.approx(rref[a], rel=1e-12, abs=1e-12)
        oref = O.distribute_observations(O.mean_std_filter(env.env.obs[0], rs, True, 10.0), spec.obs_indices)
        for a in obs:
            np.testing.assert_allclose(obs[a], oref[a], rtol=1e-12, atol=1e-12)
        assert set(done) == {"__all__"} and isinstance(done["__all__"], bool)
        assert info["reward_forward"] == fw
    env.close()


def test_host_env_thread_pool_many_small_jobs():
    """The pool under back-to-back small jobs (more threads than chunks, 3,000 jobs): a worker
    that finishes late must never run a chunk of the next job with the previous job's function
    (the generation check in hostenv::Pool::run); results equal the single-threaded env."""
    runs = []
    for threads in (8, 1):
        e = N.HostEnv(5, 43, threads, seed=3)
        e.reset()
        rng = np.random.default_rng(1)
        for _ in range(1500):
            e.act[:] = rng.uniform(-1, 1, size=(5, 8)).astype(np.float32)
            e.step(0, 2)
            e.step(2, 5)
        runs.append((e.obs.copy(), e.fw.copy()))
        e.close()
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    np.testing.assert_array_equal(runs[0][1], runs[1][1])


def test_host_env_close_drops_buffer_views_and_reset_returns_copy():
    """after close() no attribute of the HostEnv views freed pinned memory (the
    views are dropped first), further calls raise, and reset() hands out a copy -- not the
    live buffer the next step() overwrites."""
    e = N.HostEnv(4, 43, 1, seed=1)
    o = e.reset()
    e.act[:] = 0.5
    e.step()
    assert not np.array_equal(o, e.obs)      # the step changed the live buffer, not the copy
    e.close()
    assert e.obs is None and e.act is None and e.fw is None and e.cfrc is None and e.done is None
    with pytest.raises(N.DdrlError):
        e.step()
    assert np.isfinite(o).all()              # the caller's copy stays valid


def test_host_env_draws_target_velocity_per_reset_like_random_choice():
    """VERDICT r3 missing 2: every env draws its episode's target velocity from the list on each
    reset (random.choice, quantruped_adaptor_multi_environment.py:47-50, 214-216).  Over all
    episodes (the reset of every env, then every episode end) the draws follow the oracle's
    rule (every list position equally likely: oracle.target_velocity_pmf) by a chi-square test;
    a velocity changes only at an episode end; the TVel observation column and the forward
    reward use the env's own velocity (the reward against the oracle's formula per env, with
    the plain env's x velocity from a 43-column twin stepped with the same actions)."""
    from scipy import stats
    from oracle import ddrl_oracle as O
    tv_list = [0.5, 1.0, 1.0, 2.0]
    n = 192
    twin = N.HostEnv(n, 43, 2, seed=21)
    env = N.HostEnv(n, 44, 3, seed=21, target_velocity=tv_list)
    twin.reset()
    env.reset()
    tv = env.target_velocities
    draws = list(tv)
    assert np.all(env.obs[:, 43] == tv)
    rng = np.random.default_rng(8)
    n_done = 0
    for _ in range(1100):          # past the 1000-step TimeLimit: every env ends an episode
        a = rng.uniform(-1, 1, size=(n, 8)).astype(np.float32)
        twin.act[:] = a
        env.act[:] = a
        twin.step()
        env.step()
        done = env.done.astype(bool)
        np.testing.assert_array_equal(done, twin.done.astype(bool))
        np.testing.assert_allclose(env.fw, O.tvel_forward_reward(twin.fw.astype(np.float64), tv),
                                   rtol=1e-5, atol=1e-6)   # this step's reward: the episode's velocity
        new = env.target_velocities
        assert np.all(new[~done] == tv[~done])                  # no re-draw inside an episode
        draws += list(new[done])
        n_done += int(done.sum())
        tv = new
        assert np.all(env.obs[:, 43] == tv)
        np.testing.assert_array_equal(env.obs[:, :43], twin.obs)
    assert n_done >= n
    pmf = O.target_velocity_pmf(tv_list)
    vals = sorted(pmf)
    counts = np.array([np.sum(np.asarray(draws) == np.float32(v)) for v in vals])
    assert counts.sum() == len(draws)
    expected = np.array([pmf[v] for v in vals]) * len(draws)
    assert stats.chisquare(counts, expected).pvalue > 1e-3, (counts, expected)
    with pytest.raises(N.DdrlError):
        N.HostEnv(8, 44, 1, target_velocity=[1.0, 0.0])      # the TVel reward divides by it
    twin.close()
    env.close()


def test_host_env_reset_state_is_update_environment_after_epoch():
    """VERDICT r3 missing 3: update_environment_after_epoch (adaptor :97-122, run on every env
    after every iteration by train_experiment_1's on_train_result) resets the gym env: every
    env's state and TimeLimit count restart, the target velocity stays, no done flag is raised,
    and the observation buffer is untouched (the adaptor discards that observation).  Every env
    then runs the full 1000 steps to its TimeLimit (the staggered phases are gone)."""
    from ddrl_amd.hostenv import HostMultiAgentEnv
    n = 24
    env = N.HostEnv(n, 44, 2, seed=4, target_velocity=[0.5, 1.5])
    env.reset()
    rng = np.random.default_rng(1)
    for _ in range(5):
        env.act[:] = rng.uniform(-1, 1, size=(n, 8)).astype(np.float32)
        env.step()
    obs, done, tv = env.obs.copy(), env.done.copy(), env.target_velocities
    env.reset_state()
    np.testing.assert_array_equal(env.obs, obs)
    np.testing.assert_array_equal(env.done, done)
    np.testing.assert_array_equal(env.target_velocities, tv)
    env.act[:] = 0.0
    steps_to_done = np.full(n, -1)
    for k in range(1, 1001):
        env.step()
        d = env.done.astype(bool)
        steps_to_done[d & (steps_to_done < 0)] = k
    # with zero actions the stand-in torso stays up: every env reaches the TimeLimit exactly
    assert np.all(steps_to_done == 1000), steps_to_done
    env.close()
    # the dict API forwards the hook
    denv = HostMultiAgentEnv("QuantrupedMultiEnv_Local", {"target_velocity": [0.5, 1.0]}, n_envs=8, n_threads=2)
    o = denv.reset()
    assert set(np.unique(denv.target_velocities)) <= {0.5, 1.0}
    before = denv.target_velocities
    denv.update_environment_after_epoch(1000)
    np.testing.assert_array_equal(denv.target_velocities, before)
    o2, r, d, _ = denv.step({a: np.zeros((8, 2)) for a in denv.agent_names})
    assert not d["__all__"] and np.isfinite(o2["agent_FL"]).all()
    denv.close()


def test_gnn_layer_config_is_validated():
    """f4: model_config "gnn_layer" selects the message-passing layer of the graph model
    (models/graph_net.py:20 in the reference); unknown names and non-graph envs are refused."""
    from ddrl_amd.spec import make_cfg
    GNN_ENV = "QuantrupedMultiEnv_DecentralShared_Graph"
    for name, code in N.GNN_LAYERS.items():
        cfg, _ = make_cfg(GNN_ENV, 4, 2, {"model": {"custom_model": "gnn", "gnn_layer": name}})
        assert cfg.gnn_layer == code
    with pytest.raises(ValueError, match="gnn_layer"):
        make_cfg(GNN_ENV, 4, 2, {"model": {"custom_model": "gnn", "gnn_layer": "sage"}})
    with pytest.raises(ValueError, match="gnn_layer"):
        make_cfg("QuantrupedMultiEnv_Local", 4, 2, {"model": {"gnn_layer": "gat1"}})


@pytest.mark.parametrize("layer", ["mpnn", "gcn", "mpnn2", "gat1"])
def test_glorot_gnn_init_matches_oracle_per_layer(layer):
    from oracle import ddrl_oracle as O
    from ddrl_amd.models import glorot_gnn_flat
    shapes = O.gnn_param_shapes(4, layer=layer)
    ref = O.pack(O.gnn_init(np.random.default_rng(6), 4, layer=layer), shapes)
    np.testing.assert_array_equal(glorot_gnn_flat(np.random.default_rng(6), 2, layer=layer), ref)


def test_bench_parallel_mode_and_pmc_provenance():
    """bench.py's choice of multi-rank mode (round 6: gather by default for a shared policy) and
    the committed counter pass it reads its traffic / provenance figures from."""
    import bench
    assert bench.parallel_mode("auto", 4, 1) == "single"
    assert bench.parallel_mode("auto", 4, 8) == "replicas"         # Local, C3: no collective
    assert bench.parallel_mode("auto", 1, 8) == "gather"           # C4 / C5: the exact mode
    assert bench.parallel_mode("ddp", 1, 8) == "ddp"
    assert bench.parallel_mode("ddp", 4, 8) == "replicas"          # independent policies never all-reduce
    assert bench.parallel_mode("gather", 4, 2) == "gather"
    assert bench.parallel_mode("auto", 1, 1, force_ddp=True) == "ddp"
    for key, P in (("local", 4), ("c4", 1), ("c5", 1)):
        ns = bench.pmc_ns_per_step(key, P)
        assert ns is not None and 5e3 < ns < 5e4, (key, ns)      # one sequential step: 5 - 50 us
        assert bench.pmc_traffic(key, 1) > 0
    assert bench.pmc_summary("local")[1].startswith("profiles/r06")
    # the same recipe's kernel-trace pass, per sequential step (r06: Local 10.42 us, C5 16.83 us)
    assert 9e3 < bench.trace_ns_per_step("local", 64000) < 12e3
    assert 15e3 < bench.trace_ns_per_step("c5", 1) < 19e3
    assert bench.trace_ns_per_step("c5_3launch", 1) > bench.trace_ns_per_step("c5", 1)
