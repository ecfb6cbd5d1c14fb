"""Synthetic vectorized QuAntruped data, resident in HBM (SURVEY 8(d) synthetic inputs).

MuJoCo is not part of this path (and not installed); the metric is defined on synthetic
rollouts: obs ~ N(0,1)-like, noise eps ~ N(0,1), forward reward ~ N(0,1), contact forces
~ N(0,1), and episode ends every 1000 steps with staggered phases (gym TimeLimit 1000,
simulation_envs/__init__.py:27-32).
"""
from __future__ import annotations

import torch


class SyntheticRollout:
    def __init__(self, n_envs, frag_len, obs_dim, n_agents, act_dim, device, seed=0):
        g = torch.Generator(device=device)
        g.manual_seed(seed)
        T, N = frag_len, n_envs
        kw = dict(device=device, generator=g, dtype=torch.float32)
        self.obs = torch.randn((T + 1, N, obs_dim), **kw)
        self.eps = torch.randn((T, N, n_agents, act_dim), **kw)
        self.fw = torch.randn((T, N), **kw)
        self.cfrc = torch.randn((T, N, 14, 6), **kw)
        self.phase = torch.randint(0, 1000, (N,), device=device, generator=g)
        self.actions = torch.zeros((N, 8), device=device, dtype=torch.float32)
        self.T, self.N = T, N
        self.t_global = 0
        self.done = torch.zeros((T, N), dtype=torch.uint8, device=device)

    def dones_for_fragment(self):
        t = torch.arange(self.T, device=self.phase.device)[:, None] + self.t_global
        # in place: the buffer keeps its address, so the library's captured rollout graph
        # (keyed by the buffers of the call) is re-used
        self.done.copy_(((t + self.phase[None, :]) % 1000) == 999)
        self.t_global += self.T
        return self.done
