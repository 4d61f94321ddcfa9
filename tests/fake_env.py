"""A CPU stand-in with RadiotherapyVecEnv's interface, for testing the
trainer's host logic and its data-parallel path without a GPU."""
import numpy as np
import torch

from ppo_radiotherapy_amd import _lib, spaces


class FakeVecEnv:
    """obs_shape (9,): a smooth visionless toy; a 4-D obs_shape: vision-shaped
    observations (fresh uniform volumes every step) for the C3D agent.
    `reward_scale` lets data-parallel tests give ranks different advantage
    distributions (rank-local statistics then differ from the union's)."""

    def __init__(self, num_envs, seed=0, device="cpu", obs_shape=(9,), reward_scale=1.0):
        self.num_envs = num_envs
        self.device = torch.device(device)
        self.obs_shape = tuple(obs_shape)
        self.vision = len(self.obs_shape) == 4
        self.reward_scale = float(reward_scale)
        self.single_observation_space = spaces.Box(0.0, 1.0, self.obs_shape, np.float32)
        self.single_action_space = spaces.Box(-1.0, 1.0, (6,), np.float32)
        self.g = torch.Generator().manual_seed(seed)
        self.obs = torch.zeros(num_envs, *self.obs_shape)
        self.t = torch.zeros(num_envs, dtype=torch.int64)
        self.info = torch.zeros(num_envs, _lib.INFO_W)

    def reset(self, seed=None, options=None):
        self.obs = torch.rand(self.num_envs, *self.obs_shape, generator=self.g) * 2 - 1
        self.t.zero_()
        return self.obs, {}

    def step(self, actions, info_out=None):
        a = actions.clamp(-1, 1)
        if self.vision:
            self.obs = torch.rand(self.num_envs, *self.obs_shape, generator=self.g)
            reward = -(a[:, :3] ** 2).sum(1) + self.obs[:, 0].mean((1, 2, 3))
        else:
            self.obs = (self.obs * 0.9 + 0.1 * torch.cat([a, a[:, :3]], 1)).contiguous()
            reward = -(self.obs[:, :3] ** 2).sum(1)
        reward = reward * self.reward_scale
        self.t += 1
        term = self.t >= 7
        info = self.info if info_out is None else info_out
        info.zero_()
        info[:, 0] = reward
        info[:, 16] = 1.0
        info[:, 17] = term.float()
        info[:, 18] = reward * 7
        info[:, 19] = 7.0
        self.t[term] = 0
        return self.obs, reward, term, torch.zeros_like(term), {}


def torch_gae(tr, next_value):
    """train.py:163-181 verbatim, as the CPU reference for rt_gae."""
    cfg = tr.cfg
    last = 0
    for t in reversed(range(tr.T)):
        if t == tr.T - 1:
            nnt, nv = 1.0 - tr.next_done, next_value
        else:
            nnt, nv = 1.0 - tr.dones[t + 1], tr.values[t + 1]
        delta = tr.rewards[t] + cfg.gamma * nv * nnt - tr.values[t]
        tr.advantages[t] = last = delta + cfg.gamma * cfg.gae_lambda * nnt * last
    tr.returns.copy_(tr.advantages + tr.values)
