"""Host-side mirror of the reference's `simulation_envs` plugin surface.

Reference: simulation_envs/__init__.py:53-67 (register_env names),
quantruped_adaptor_multi_environment.py:8-272 (QuantrupedMultiPoliciesEnv), and the
env classes in quantruped_{fourDecentralizedController, singleDecentralizedController,
twoDecentralizedController, GraphDecentralizedController, centralizedController}_*.py.

Each class keeps the reference's class attributes (`policy_names`, `agent_names`), the
static `return_policies(use_target_velocity)` and `policy_mapping_fn(agent_id)`, and the
per-agent tables (`obs_indices`, `action_indices`, `contact_force_indices`).  The physics
(MuJoCo) is not part of this path: the vectorized environments that feed the HIP kernels
live in `ddrl_amd.envs`, and the tables below become the kernels' routing configuration
through `ddrl_amd.spec.make_cfg`.
"""
from __future__ import annotations

from ..spaces import Box, MultiDiscrete, Tuple
from . import layouts
from .layouts import (get_action_indices, get_contact_force_indices, get_obs_indices)

LEGS = ("fl", "hl", "hr", "fr")
LEG_AGENTS = ["agent_FL", "agent_HL", "agent_HR", "agent_FR"]


class QuantrupedMultiPoliciesEnv:
    """Base class (quantruped_adaptor_multi_environment.py:8-272): central policy."""

    policy_names = ["centr_A_policy"]
    agent_names = ["central_agent"]
    model_kind = "ffn"

    def __init__(self, config=None):
        config = dict(config or {})
        self.config = config
        self.ctrl_cost_weight = config.get("ctrl_cost_weight", 0.5)
        self.contact_cost_weight = config.get("contact_cost_weight", 5e-4)
        self.hf_smoothness = config.get("hf_smoothness", 1.0)
        self.target_velocity_list = config.get("target_velocity")
        self.use_target_velocity = self.target_velocity_list is not None
        if self.use_target_velocity and not isinstance(self.target_velocity_list, (list, tuple)):
            self.target_velocity_list = [self.target_velocity_list]   # adaptor :47-49
        if config.get("global_reward", False):
            self.reward_mode = "global"
        elif config.get("norm_reward", False):
            self.reward_mode = "norm"
        else:
            self.reward_mode = "per_leg"
        self.curriculum_learning = config.get("curriculum_learning", False)
        self._init_tables()

    # -- tables --------------------------------------------------------------------
    def _init_tables(self):
        self.obs_indices = {"central_agent": get_obs_indices(None, self.obs_fields)}
        self.action_indices = {"central_agent": get_action_indices(None)}
        self.contact_force_indices = {"central_agent": get_contact_force_indices(None)}

    @property
    def obs_fields(self):
        return layouts.TVEL_OBS_FIELDS if self.use_target_velocity else layouts.OBS_FIELDS

    @property
    def _agent_ids(self):
        return set(self.agent_names)

    @staticmethod
    def policy_mapping_fn(agent_id):
        return QuantrupedMultiPoliciesEnv.policy_names[0]

    @staticmethod
    def return_policies(use_target_velocity=False):
        n = 43 + use_target_velocity
        return {QuantrupedMultiPoliciesEnv.policy_names[0]:
                (None, Box(-float("inf"), float("inf"), (n,), "float64"), Box(-1.0, 1.0, (8,)), {})}

    def update_environment_after_epoch(self, timesteps_total):
        """Curriculum hook (adaptor :97-122), the spec's part: update_after_epoch.  The env
        reset that follows it in the reference is the backend's (HostMultiAgentEnv /
        ddrl_amd.envs backends: every env's state and TimeLimit count restart); terrain
        regeneration is MuJoCo-side and out of scope."""
        self.update_after_epoch(timesteps_total)

    def update_after_epoch(self, timesteps_total):
        pass


def _four_leg_tables(self, obs_prefixes):
    self.obs_indices = {a: get_obs_indices(p, self.obs_fields) for a, p in zip(LEG_AGENTS, obs_prefixes)}
    self.action_indices = {a: get_action_indices([leg]) for a, leg in zip(LEG_AGENTS, LEGS)}
    self.contact_force_indices = {a: get_contact_force_indices(['body', leg], weights=[1. / 4., 1.])
                                  for a, leg in zip(LEG_AGENTS, LEGS)}


def _leg_policies(names, n_dims):
    obs = Box(-float("inf"), float("inf"), (n_dims,), "float64")
    return {p: (None, obs, Box(-1.0, 1.0, (2,)), {}) for p in names}


class QuantrupedFourControllerSuperEnv(QuantrupedMultiPoliciesEnv):
    """quantruped_fourDecentralizedController_environments.py:6-48"""
    policy_names = ["policy_FL", "policy_HL", "policy_HR", "policy_FR"]
    agent_names = list(LEG_AGENTS)
    obs_prefixes = [['body', 'fl'], ['body', 'hl'], ['body', 'hr'], ['body', 'fr']]
    base_dims = 19

    def _init_tables(self):
        _four_leg_tables(self, self.obs_prefixes)

    @staticmethod
    def policy_mapping_fn(agent_id):
        if agent_id.startswith("agent_FL"):
            return "policy_FL"
        elif agent_id.startswith("agent_HL"):
            return "policy_HL"
        elif agent_id.startswith("agent_HR"):
            return "policy_HR"
        return "policy_FR"

    @classmethod
    def return_policies(cls, use_target_velocity=False):
        return _leg_policies(cls.policy_names, cls.base_dims + use_target_velocity)


class QuantrupedFullyDecentralizedEnv(QuantrupedFourControllerSuperEnv):
    """:168-225 -- each leg sees only itself (d = 19)."""


class Quantruped_LocalSingleNeighboringLeg_Env(QuantrupedFourControllerSuperEnv):
    """:227-291 -- plus the counter-clockwise neighbour (d = 27)."""
    obs_prefixes = [['body', 'fl', 'hl'], ['body', 'hl', 'hr'], ['body', 'hr', 'fr'], ['body', 'fr', 'fl']]
    base_dims = 27


class Quantruped_LocalSingleDiagonalLeg_Env(QuantrupedFourControllerSuperEnv):
    """:293-356 -- plus the diagonal leg (HR reuses FL's table, FR reuses HL's: :336-339)."""
    obs_prefixes = [['body', 'fl', 'hr'], ['body', 'hl', 'fr'], ['body', 'fl', 'hr'], ['body', 'hl', 'fr']]
    base_dims = 27


class Quantruped_LocalSingleToFront_Env(QuantrupedFourControllerSuperEnv):
    """:358-423"""
    obs_prefixes = [['body', 'fl', 'hl'], ['body', 'hl', 'hr'], ['body', 'hr', 'hl'], ['body', 'fr', 'hr']]
    base_dims = 27


class Quantruped_Local_Env(QuantrupedFourControllerSuperEnv):
    """:425-488 -- plus both neighbouring legs (d = 35); the headline configuration."""
    obs_prefixes = [['body', 'fl', 'hl', 'fr'], ['body', 'hl', 'hr', 'fl'],
                    ['body', 'hr', 'fr', 'hl'], ['body', 'fr', 'fl', 'hr']]
    base_dims = 35


class QuantrupedFullyDecentralizedGlobalCostEnv(QuantrupedFullyDecentralizedEnv):
    """quantruped_fourDecentralizedController_GlobalCosts_environments.py: the same routing
    with the global reward (the reference's own distribute_reward there is broken, see
    SURVEY Appendix B; the global-reward formula of the adaptor is used)."""

    def __init__(self, config=None):
        config = dict(config or {})
        config["global_reward"] = True
        super().__init__(config)


class QuantrupedSingleControllerSuperEnv(QuantrupedMultiPoliciesEnv):
    """quantruped_singleDecentralizedController_environments.py:6-59 -- one shared policy."""
    policy_names = ["policy_legs"]
    agent_names = list(LEG_AGENTS)

    def _init_tables(self):
        _four_leg_tables(self, [['body', leg] for leg in LEGS])

    @staticmethod
    def policy_mapping_fn(agent_id):
        return QuantrupedSingleControllerSuperEnv.policy_names[0]

    @staticmethod
    def return_policies(use_target_velocity=False):
        return _leg_policies(QuantrupedSingleControllerSuperEnv.policy_names, 19 + use_target_velocity)


class QuantrupedSingleDecentralizedEnv(QuantrupedSingleControllerSuperEnv):
    pass


class QuantrupedSingleDecentralizedLegIDEnv(QuantrupedSingleControllerSuperEnv):
    """quantruped_singleDecentralizedController_environments.py:66-114: every agent
    receives (leg index, 19 normalized features).  RLlib's Tuple preprocessor one-hot
    encodes the MultiDiscrete part, so the model input is one_hot(index, 4) ++ features
    (d = 23): `policy_obs_indices` encodes the one-hot as the constants -1 (0.0) and -2
    (1.0) of the gather table."""
    leg_angles = {'agent_FL': 45., 'agent_HL': 135., 'agent_HR': -135., 'agent_FR': -45.}
    leg_index_obs = True   # (leg index, features): the "cup" model consumes the tuple as is

    def _init_tables(self):
        super()._init_tables()
        self.policy_obs_indices = {a: [-2 if k == j else -1 for k in range(4)] + list(self.obs_indices[a])
                                   for j, a in enumerate(self.agent_names)}

    @staticmethod
    def return_policies(use_target_velocity=False):
        obs = Box(-float("inf"), float("inf"), (19 + use_target_velocity,), "float64")
        space = Tuple([MultiDiscrete([4]), obs])
        return {QuantrupedSingleControllerSuperEnv.policy_names[0]: (None, space, Box(-1.0, 1.0, (2,)), {})}


class QuantrupedSingleDecentralizedLegTransforms(QuantrupedSingleControllerSuperEnv):
    """quantruped_singleDecentralizedController_environments.py:117-148: the observation
    scale is all ones (no-op); concatenate_actions negates the fr_knee and hr_knee actions
    of the env action vector (`action_negate`).  Rewards use the agents' own actions, whose
    squares the sign does not change."""

    def _init_tables(self):
        super()._init_tables()
        neg = set(get_action_indices(['fr_knee']) + get_action_indices(['hr_knee']))
        self.action_negate = {a: [i in neg for i in self.action_indices[a]] for a in self.agent_names}


class QuantrupedTwoControllerSuperEnv(QuantrupedMultiPoliciesEnv):
    """quantruped_twoDecentralizedController_environments.py (A = 4, d = 27)."""
    groups = (('fl', 'hl'), ('hr', 'fr'))

    def _init_tables(self):
        self.obs_indices, self.action_indices, self.contact_force_indices = {}, {}, {}
        for a, g in zip(self.agent_names, self.groups):
            self.obs_indices[a] = get_obs_indices(['body', *g], self.obs_fields)
            self.action_indices[a] = get_action_indices(list(g))
            self.contact_force_indices[a] = get_contact_force_indices(['body', *g], weights=[1. / 2., 1., 1.])

    @classmethod
    def return_policies(cls, use_target_velocity=False):
        obs = Box(-float("inf"), float("inf"), (27 + use_target_velocity,), "float64")
        return {p: (None, obs, Box(-1.0, 1.0, (4,)), {}) for p in cls.policy_names}


class Quantruped_TwoSideControllers_Env(QuantrupedTwoControllerSuperEnv):
    policy_names = ["policy_LEFT", "policy_RIGHT"]
    agent_names = ["agent_LEFT", "agent_RIGHT"]

    @staticmethod
    def policy_mapping_fn(agent_id):
        return "policy_LEFT" if agent_id.startswith("agent_LEFT") else "policy_RIGHT"


class Quantruped_TwoDiagControllers_Env(QuantrupedTwoControllerSuperEnv):
    policy_names = ["policy_FLHR", "policy_HLFR"]
    agent_names = ["agent_FLHR", "agent_HLFR"]
    groups = (('fl', 'hr'), ('hl', 'fr'))

    @staticmethod
    def policy_mapping_fn(agent_id):
        return "policy_FLHR" if agent_id.startswith("agent_FLHR") else "policy_HLFR"


class Quantruped_Centralized_Env(QuantrupedMultiPoliciesEnv):
    """quantruped_centralizedController_environment.py:6-74.  The reference keys
    return_policies by the base class's "centr_A_policy" while its mapping function returns
    "central_policy" (SURVEY Appendix B.2); the published checkpoints use
    "central_policy", so both name the one central policy here."""
    policy_names = ["central_policy"]
    agent_names = ["central_agent"]

    @staticmethod
    def policy_mapping_fn(agent_id):
        return "central_policy"

    @staticmethod
    def return_policies(use_target_velocity=False):
        n = 43 + use_target_velocity
        return {"central_policy": (None, Box(-float("inf"), float("inf"), (n,), "float64"),
                                   Box(-1.0, 1.0, (8,)), {})}


class QuantrupedDecentralizedSharedGraphEnv(QuantrupedMultiPoliciesEnv):
    """quantruped_GraphDecentralizedController_environments.py:123-245: one shared
    `leg_policy`; every agent receives (node_idx, X[4, 23], adj[4, 4]) where
    X[n] = normalized 19 leg features ++ ego quaternion (leg_encoding_ego)."""
    policy_names = ["leg_policy"]
    agent_names = list(LEG_AGENTS)
    model_kind = "gnn"
    leg_angles = {'agent_FL': 45., 'agent_HL': 135., 'agent_HR': -135., 'agent_FR': -45.}

    def _init_tables(self):
        _four_leg_tables(self, [['body', leg] for leg in LEGS])
        self.adj = self.create_adj()

    def create_edge_index(self):
        idx = self.agent_names.index
        e = lambda s, r: [idx(s), idx(r)]
        return [e('agent_FL', 'agent_HL'), e('agent_HL', 'agent_HR'), e('agent_HR', 'agent_FR'),
                e('agent_FR', 'agent_FL'), e('agent_HL', 'agent_FL'), e('agent_HR', 'agent_HL'),
                e('agent_FR', 'agent_HR'), e('agent_FL', 'agent_FR')]

    def create_adj(self):
        adj = [[0.0] * 4 for _ in range(4)]
        for s, r in self.create_edge_index():
            adj[s][r] = 1.0
        return adj

    @staticmethod
    def policy_mapping_fn(agent_id):
        return 'leg_policy'

    @staticmethod
    def return_policies(use_target_velocity=False):
        n = 19 + use_target_velocity + 2 + 2
        space = Tuple([MultiDiscrete([4]), Box(-float("inf"), float("inf"), (4, n), "float64"),
                       MultiDiscrete([[2] * 4] * 4)])
        return {"leg_policy": (None, space, Box(-1.0, 1.0, (2,)), {})}


class QuantrupedDecentralizedGraphEnv(QuantrupedFourControllerSuperEnv):
    """quantruped_GraphDecentralizedController_environments.py:37-121: four policies with
    19-d graph nodes.  The GraphNet ("gnn") needs 23-d nodes (19 features + the ego
    quaternion of its hypernetwork), so this env has no consistent model pairing in the
    reference; it is registered and refuses to build a context."""
    model_kind = "gnn-19"


# register_env names (simulation_envs/__init__.py:53-67).  The reference registers
# "QuantrupedMultiEnv_Centralized" to the base class (Appendix B.2); it maps to the
# working centralized env here.
ENV_REGISTRY = {
    "QuantrupedMultiEnv_Centralized": Quantruped_Centralized_Env,
    "QuantrupedMultiEnv_DecentralShared_Graph": QuantrupedDecentralizedSharedGraphEnv,
    "QuantrupedMultiEnv_FullyDecentral": QuantrupedFullyDecentralizedEnv,
    "QuantrupedMultiEnv_FullyDecentralGlobalCost": QuantrupedFullyDecentralizedGlobalCostEnv,
    "QuantrupedMultiEnv_SingleNeighbor": Quantruped_LocalSingleNeighboringLeg_Env,
    "QuantrupedMultiEnv_SingleDiagonal": Quantruped_LocalSingleDiagonalLeg_Env,
    "QuantrupedMultiEnv_SingleToFront": Quantruped_LocalSingleToFront_Env,
    "QuantrupedMultiEnv_Local": Quantruped_Local_Env,
    "QuantrupedMultiEnv_TwoSides": Quantruped_TwoSideControllers_Env,
    "QuantrupedMultiEnv_TwoDiags": Quantruped_TwoDiagControllers_Env,
    "QuantrupedMultiEnv_SharedDecentral": QuantrupedSingleDecentralizedEnv,
    "QuantrupedMultiEnv_SharedDecentralLegID": QuantrupedSingleDecentralizedLegIDEnv,
    "QuantrupedMultiEnv_SharedDecentralLegTransforms": QuantrupedSingleDecentralizedLegTransforms,
    "QuantrupedMultiEnv_Decentral_Graph": QuantrupedDecentralizedGraphEnv,
}


def register_env(name, creator):
    ENV_REGISTRY[name] = creator


def get_env_class(name):
    try:
        return ENV_REGISTRY[name]
    except KeyError:
        raise KeyError(f"unknown env {name!r}; registered: {sorted(ENV_REGISTRY)}") from None
