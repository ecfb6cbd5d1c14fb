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

    def update_environment_after_epoch(self, timesteps_total):
        """env.reset() of every env (quantruped_adaptor_multi_environment.py:97-122): the
        TimeLimit counts restart; no done flag, the next observation is the usual draw."""
        self.t.zero_()


class HostVecEnv:
    """The host env plane (ddrl_amd.native.HostEnv: the QuAntruped stand-in stepped by a pool of
    host threads into pinned buffers) as a trainer backend: device tensors in and out, with a
    per-env target velocity drawn from the list on every reset (TVel envs) and the
    update_environment_after_epoch reset.  The bench's PCIe leg uses the same plane through
    the pipelined ddrl_rollout_hostenv instead."""

    def __init__(self, n_envs, obs_dim, device, seed=0, n_threads=4, target_velocity=0.0):
        import torch
        from .native import HostEnv
        self.torch, self.device = torch, device
        self.env = HostEnv(n_envs, obs_dim, n_threads, seed, target_velocity)

    def _dev(self, a):
        return self.torch.from_numpy(a).to(self.device, non_blocking=False)

    def reset(self):
        return self._dev(self.env.reset())

    def step(self, actions):
        self.env.act[:] = actions.detach().to("cpu").numpy()
        self.env.step()
        return (self._dev(self.env.obs.copy()), self._dev(self.env.fw.copy()), self._dev(self.env.cfrc.copy()),
                self._dev(self.env.done.copy()))

    def update_environment_after_epoch(self, timesteps_total):
        self.env.reset_state()

    @property
    def target_velocities(self):
        return self.env.target_velocities

    def close(self):
        self.env.close()
