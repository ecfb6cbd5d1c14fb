"""The reference's MultiAgentEnv surface over the host env plane (f1).

RLlib callers that step environments one action dict at a time -- the evaluation scripts
(evaluation/evaluate_trained_policies_pd.py), a custom sampler -- use
`QuantrupedMultiPoliciesEnv.reset() -> {agent_id: obs}` and
`step({agent_id: action}) -> (obs_dict, rew_dict, {"__all__": done}, info)`
(simulation_envs/quantruped_adaptor_multi_environment.py:214-250).  `HostMultiAgentEnv` gives
that surface for any registered env name, over the C++ host env plane (ddrl_amd.native.HostEnv:
the QuAntruped stand-in stepped by host threads): the env-side MeanStdFilter (RunningStat push
per env, then (x - mean) / (std + 1e-8) clipped to +-10, observation_filter.py:3-12 and
adaptor :83-85), `distribute_observations` (:124-136), `concatenate_actions` (:205-212) and the
per-leg / global / normalized rewards (:160-203) are the env's own host-side work, as in the
reference.  The training hot path does not come through here: the trainer and the bench run
the vectorized rollout on the device (ddrl_rollout_fragment / ddrl_rollout_hostenv).

With n_envs > 1 every value is batched over the envs: obs_dict[agent] is [n_envs, d],
rewards [n_envs], dones {"__all__": all envs done, "envs": [n_envs] flags}.
"""
from __future__ import annotations

import numpy as np

from . import native as N
from .simulation_envs import get_env_class


class HostMultiAgentEnv:
    def __init__(self, env, config=None, n_envs=1, n_threads=1, seed=0, filter_clip=10.0):
        cls = get_env_class(env) if isinstance(env, str) else env
        self.spec = cls(dict(config or {}))
        if self.spec.model_kind != "ffn":
            raise ValueError(f"{cls.__name__}: the dict API covers the fcnet envs (per-agent observation vectors)")
        self.agent_names = list(self.spec.agent_names)
        self.n = int(n_envs)
        self.D = len(self.spec.obs_fields)
        tv = self.spec.target_velocity_list
        # every env draws random.choice(target_velocity_list) on each reset
        # (quantruped_adaptor_multi_environment.py:47-50, :214-216), in the env plane
        self.env = N.HostEnv(self.n, self.D, n_threads, seed, [float(v) for v in tv] if tv else 0.0)
        self.clip = filter_clip
        # env-side MeanStdFilter singleton: RunningStat (n, M, S), fp64
        self.rs_n, self.rs_M, self.rs_S = 0, np.zeros(self.D), np.zeros(self.D)
        self.obs_idx = {a: np.asarray(self.spec.obs_indices[a]) for a in self.agent_names}
        self.act_idx = {a: np.asarray(self.spec.action_indices[a]) for a in self.agent_names}
        neg = getattr(self.spec, "action_negate", {})
        self.act_sign = {a: np.where(np.asarray(neg.get(a, [False] * len(self.act_idx[a]))), -1.0, 1.0)
                         for a in self.agent_names}
        self.contact = {a: tuple(np.asarray(x) for x in self.spec.contact_force_indices[a]) for a in self.agent_names}
        self.last_actions = np.zeros((self.n, 8))

    # -- observation side (adaptor :83-85, :124-136) ------------------------------------
    def _normalize(self, obs):
        out = np.empty((self.n, self.D))
        for e in range(self.n):          # RunningStat.push row by row, then normalize the row
            x = np.asarray(obs[e], np.float64)
            self.rs_n += 1
            if self.rs_n == 1:
                self.rs_M[:] = x
            else:
                d = x - self.rs_M
                self.rs_M += d / self.rs_n
                self.rs_S += d * d * (self.rs_n - 1) / self.rs_n
            var = self.rs_S / (self.rs_n - 1) if self.rs_n > 1 else np.square(self.rs_M)
            z = (x - self.rs_M) / (np.sqrt(var) + 1e-8)
            out[e] = np.clip(z, -self.clip, self.clip) if self.clip else z
        return out

    def _distribute(self, z):
        ext = np.concatenate([z, np.zeros((self.n, 1)), np.ones((self.n, 1))], 1)   # LegID constants -1 / -2
        col = lambda i: i if i >= 0 else self.D + (-1 - i)
        obs = {}
        for a in self.agent_names:
            v = ext[:, [col(int(i)) for i in self.obs_idx[a]]]
            obs[a] = v[0] if self.n == 1 else v
        return obs

    def reset(self):
        """{agent_id: observation} of freshly reset envs (adaptor :214-218)."""
        return self._distribute(self._normalize(self.env.reset()))

    # -- action / reward side (adaptor :160-212) -----------------------------------------
    def _concatenate_actions(self, action_dict):
        act = np.zeros((self.n, 8))
        for a in self.agent_names:
            v = np.asarray(action_dict[a], np.float64).reshape(self.n, -1)
            act[:, self.act_idx[a]] = np.clip(v, -1.0, 1.0) * self.act_sign[a]
        return act

    def _rewards(self, fw, cfrc, act):
        cf = np.clip(np.asarray(cfrc, np.float64), -1.0, 1.0)
        na = len(self.agent_names)
        w_ctrl, w_cont = self.spec.ctrl_cost_weight, self.spec.contact_cost_weight
        fw = np.asarray(fw, np.float64)
        if self.spec.reward_mode == "global":
            r = (fw - w_ctrl * np.sum(act * act, 1) - w_cont * np.sum(cf * cf, (1, 2))) / na
            return {a: r for a in self.agent_names}
        out = {}
        for a in self.agent_names:
            ctrl = np.sum(act[:, self.act_idx[a]] ** 2, 1)
            idx, wts = self.contact[a]
            contact = np.zeros(self.n)
            for i, wt in zip(idx, wts):
                contact += w_cont * np.sum(cf[:, int(i)] ** 2, 1) * wt
            out[a] = fw - na * (w_ctrl * ctrl + contact) if self.spec.reward_mode == "norm" \
                else fw / na - w_ctrl * ctrl - contact
        return out

    def step(self, action_dict):
        """(obs_dict, reward_dict, {"__all__": done}, info) of one env step (adaptor :220-250).
        A done env is reset by the env plane at once; its next observation is the reset one."""
        act = self._concatenate_actions(action_dict)
        self.env.act[:] = act.astype(np.float32)
        self.env.step()
        act32 = self.env.act.astype(np.float64)     # the actions the env applied (fp32 buffer)
        rew = self._rewards(self.env.fw, self.env.cfrc, act32)
        obs = self._distribute(self._normalize(self.env.obs))
        done = self.env.done.astype(bool)
        if self.n == 1:
            rew = {a: float(r[0]) for a, r in rew.items()}
            dones = {"__all__": bool(done[0])}
        else:
            dones = {"__all__": bool(done.all()), "envs": done.copy()}
        info = {"reward_forward": self.env.fw.copy() if self.n > 1 else float(self.env.fw[0])}
        return obs, rew, dones, info

    def update_environment_after_epoch(self, timesteps_total):
        """The curriculum hook RLlib calls on every env after each training iteration
        (on_train_result, train_experiment_1_architecture_on_flat.py:171-178; adaptor :97-122):
        the spec's update_after_epoch, then env.reset() of every env (state and TimeLimit count
        restart, target velocity kept, the observation of that reset discarded).  The terrain
        regeneration (create_new_random_hfield) is MuJoCo-side and out of scope."""
        self.spec.update_after_epoch(timesteps_total)
        self.env.reset_state()

    @property
    def target_velocities(self):
        """Each env's current target velocity (TVel envs)."""
        return self.env.target_velocities

    def close(self):
        self.env.close()
