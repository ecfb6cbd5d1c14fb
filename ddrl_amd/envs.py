"""Vectorized environment backends that feed the HIP rollout kernels.

SyntheticVecEnv is the synthetic QuAntruped used for the metric (MuJoCo is out of scope
and not installed): observations and rewards are seeded Gaussian draws generated on the
device each step, contact forces likewise, and episodes end every 1000 steps with
staggered phases (the gym TimeLimit of simulation_envs/__init__.py:27-32).  A MuJoCo
backend only has to implement the same reset()/step() on host cores and hand over pinned
buffers.
"""
from __future__ import annotations


class SyntheticVecEnv:
    def __init__(self, n_envs, obs_dim, device, seed=0, max_episode_steps=1000):
        import torch
        self.torch = torch
        self.N, self.D, self.device = n_envs, obs_dim, device
        self.gen = torch.Generator(device=device)
        self.gen.manual_seed(seed)
        self.max_steps = max_episode_steps
        self.t = torch.randint(0, max_episode_steps, (n_envs,), device=device, generator=self.gen)

    def _randn(self, *shape):
        return self.torch.randn(shape, device=self.device, generator=self.gen)

    def reset(self):
        return self._randn(self.N, self.D)

    def step(self, actions):
        self.t += 1
        done = (self.t % self.max_steps == 0).to(self.torch.uint8)
        obs = self._randn(self.N, self.D)
        return obs, self._randn(self.N), self._randn(self.N, 14, 6), done
