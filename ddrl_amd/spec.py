"""Turn an env class + RLlib-style config into the C-ABI configuration (ddrl_cfg).

Config keys follow train_experiment_1_architecture_on_flat.py:96-168 and the recorded
params.json (gamma, lambda, clip_param, vf_clip_param, vf_loss_coeff, entropy_coeff, lr,
grad_clip, sgd_minibatch_size, num_sgd_iter, rollout_fragment_length, env_config{...}).
"""
from __future__ import annotations

from . import native as N
from .simulation_envs import get_env_class

PPO_DEFAULTS = {
    # RLlib 1.0 PPO defaults as recorded in the reference's params.json, overridden by the
    # exp-1 script (train_batch_size 16000, sgd_minibatch_size 128, lr 3e-4, grad_clip 0.5)
    "gamma": 0.99, "lambda": 0.95, "clip_param": 0.2, "vf_clip_param": 10.0,
    "vf_loss_coeff": 0.5, "entropy_coeff": 0.0, "kl_coeff": 0.2, "kl_target": 0.01,
    "lr": 3e-4, "grad_clip": 0.5, "sgd_minibatch_size": 128, "num_sgd_iter": 10,
    "train_batch_size": 16000, "rollout_fragment_length": 200, "shuffle_sequences": True,
    "clip_actions": True, "vf_clip_mode": "ray10",
    # RLlib-side per-policy filter: exp-1 in the fork uses NoFilter (train_experiment_1:128);
    # the published runs and the shared-policy script use MeanStdFilter (P_Local:139)
    "observation_filter": "NoFilter",
}
ENV_DEFAULTS = {"ctrl_cost_weight": 0.5, "contact_cost_weight": 5e-2, "hf_smoothness": 1.0,
                "norm_reward": False, "global_reward": False, "filter_clip": 10.0,
                "observation_filter_env": True}


def make_cfg(env, n_envs, frag_len=None, config=None):
    """env: registered name, class or instance.  Returns (DdrlCfg, env_instance)."""
    config = {**PPO_DEFAULTS, **(config or {})}
    env_config = {**ENV_DEFAULTS, **config.get("env_config", {})}
    if isinstance(env, str):
        env = get_env_class(env)
    inst = env(env_config) if isinstance(env, type) else env
    custom_model = (config.get("model") or {}).get("custom_model")
    # "cup" (models/coupling_net_glorot_uniform_init.py:32-137) takes the LegID env's
    # (leg index, features) tuple: the features are the model input and the index selects
    # the coupling row, so the model reads obs_indices (no one-hot columns)
    cup = custom_model == "cup"
    if cup and not getattr(inst, "leg_index_obs", False):
        raise ValueError(f"custom_model 'cup' needs an env whose observation is (leg index, features) "
                         f"(QuantrupedMultiEnv_SharedDecentralLegID); got {type(inst).__name__}")
    if inst.model_kind not in ("ffn", "gnn"):
        raise ValueError(f"{type(inst).__name__}: no model of the reference fits this env's observations "
                         "(SURVEY Appendix B.8)")
    agents = list(inst.agent_names)
    policies = list(type(inst).policy_names)
    mapping = type(inst).policy_mapping_fn
    c = N.DdrlCfg()
    c.n_envs = int(n_envs)
    c.frag_len = int(frag_len or config["rollout_fragment_length"])
    c.obs_full_dim = len(inst.obs_fields)
    c.n_agents = len(agents)
    c.n_policies = len(policies)
    c.model_kind = N.MODEL_GNN if inst.model_kind == "gnn" else N.MODEL_FFN
    c.act_dim = len(inst.action_indices[agents[0]])
    for j, a in enumerate(agents):
        p = policies.index(mapping(a))
        c.agent_policy[j] = p
        idx = (inst.obs_indices if cup else getattr(inst, "policy_obs_indices", inst.obs_indices))[a]
        c.obs_dim[p] = len(idx)
        for f, i in enumerate(idx):
            c.obs_index[j][f] = i
        for k, i in enumerate(inst.action_indices[a]):
            c.act_index[j][k] = i
            c.act_negate[j][k] = int(getattr(inst, "action_negate", {}).get(a, [False] * 8)[k])
        ci, cw = inst.contact_force_indices[a]
        c.n_contact[j] = len(ci)
        for k, (i, w) in enumerate(zip(ci, cw)):
            c.contact_index[j][k] = i
            c.contact_weight[j][k] = float(w[0] if isinstance(w, (list, tuple)) else w)
    if inst.model_kind == "gnn":
        for j, a in enumerate(agents):
            c.leg_angle_deg[j] = inst.leg_angles[a]
    c.filter_enabled = 1 if env_config.get("observation_filter_env", True) else 0
    c.filter_update = 1
    c.filter_clip = float(env_config.get("filter_clip", 10.0))
    c.reward_mode = {"per_leg": N.REWARD_PER_LEG, "global": N.REWARD_GLOBAL,
                     "norm": N.REWARD_NORM}[inst.reward_mode]
    c.ctrl_cost_weight = float(env_config["ctrl_cost_weight"])
    c.contact_cost_weight = float(env_config["contact_cost_weight"])
    c.gamma = config["gamma"]
    c.lambda_ = config["lambda"]
    c.clip_param = config["clip_param"]
    c.vf_clip_param = config["vf_clip_param"]
    c.vf_loss_coeff = config["vf_loss_coeff"]
    c.entropy_coeff = config["entropy_coeff"]
    c.lr = config["lr"]
    c.grad_clip = config["grad_clip"] if config["grad_clip"] is not None else 1e30
    c.adam_beta1, c.adam_beta2, c.adam_eps = 0.9, 0.999, 1e-8
    c.vf_clip_mode = N.VF_CLIP_RAY10 if config["vf_clip_mode"] == "ray10" else N.VF_CLIP_SQUARED
    c.sgd_minibatch_size = int(config["sgd_minibatch_size"])
    c.num_sgd_iter = int(config["num_sgd_iter"])
    if config["observation_filter"] not in ("NoFilter", "MeanStdFilter"):
        raise ValueError(f"observation_filter {config['observation_filter']!r} is not supported")
    c.policy_filter = 1 if config["observation_filter"] == "MeanStdFilter" else 0
    c.leg_coupling = 1 if cup else 0
    # "gnn_layer" (model_config; an extension): the message-passing layer the reference selects by
    # editing models/graph_net.py:20 -- "mpnn" (its default), "gcn", "mpnn2" or "gat1"
    layer = (config.get("model") or {}).get("custom_model_config", {}).get(
        "gnn_layer", (config.get("model") or {}).get("gnn_layer", "mpnn"))
    if layer not in N.GNN_LAYERS:
        raise ValueError(f"gnn_layer {layer!r}: one of {sorted(N.GNN_LAYERS)}")
    if layer != "mpnn" and inst.model_kind != "gnn":
        raise ValueError(f"gnn_layer {layer!r} needs the graph env / 'gnn' model")
    c.gnn_layer = N.GNN_LAYERS[layer]
    return c, inst
