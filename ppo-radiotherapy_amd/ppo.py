"""PPO trainer (reference: train.py:91-282, CleanRL continuous PPO).

Same algorithm, same config keys, same losses; re-organised for a
device-resident env:

* rollout: policy forward, Gaussian sample and the HIP env step all stay on the
  GPU; no host sync per step (the reference copies actions D2H and
  obs/rewards H2D every step, train.py:151-158).  Episode statistics are
  accumulated from the env's info rows and reduced once per iteration.
* GAE: one HIP lane per env (rt_gae), the reference's reversed loop.
* update: epochs x minibatches, minibatch indices from a device randperm
  (the reference shuffles with np.random on the host, train.py:195).
* data parallel (one process per GPU): envs are sharded, the gradient lives
  in one flat bucket that every param.grad views, and is all-reduced once per
  optimizer step (RCCL) before clip_grad_norm_, so all ranks clip the same
  global gradient; advantage normalisation uses global minibatch statistics.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass

import numpy as np
import torch
import torch.distributed as dist
from torch import nn

from . import _lib


@dataclass
class IterStats:
    """Per-iteration scalars (the reference's TensorBoard tags, train.py:42-88)."""
    episodes: int = 0
    episodic_return: float = float("nan")
    episodic_length: float = float("nan")
    tumour_reward: float = float("nan")
    lung_reward: float = float("nan")
    distance_reward: float = float("nan")
    total_reward: float = float("nan")
    value_loss: float = float("nan")
    policy_loss: float = float("nan")
    entropy: float = float("nan")
    old_approx_kl: float = float("nan")
    approx_kl: float = float("nan")
    clipfrac: float = float("nan")
    explained_variance: float = float("nan")
    learning_rate: float = float("nan")
    rollout_s: float = 0.0
    update_s: float = 0.0


class PPOTrainer:
    def __init__(self, cfg, env, agent: nn.Module, device, rank: int = 0, world: int = 1,
                 generator: torch.Generator | None = None, gae_fn=None):
        """`gae_fn(trainer, next_value)` replaces the rt_gae kernel (tests run
        the trainer on CPU with a torch reference GAE)."""
        self.cfg = cfg
        self.gae_fn = gae_fn
        self.env = env
        self.agent = agent
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        self.gen = generator
        N, T = env.num_envs, int(cfg.num_steps)
        self.N, self.T = N, T
        obs_shape = env.single_observation_space.shape
        act_shape = env.single_action_space.shape
        kw = dict(device=self.device)
        self.obs = torch.zeros((T, N, *obs_shape), **kw)
        self.actions = torch.zeros((T, N, *act_shape), **kw)
        self.logprobs = torch.zeros((T, N), **kw)
        self.rewards = torch.zeros((T, N), **kw)
        self.dones = torch.zeros((T, N), **kw)
        self.values = torch.zeros((T, N), **kw)
        self.infos = torch.zeros((T, N, _lib.INFO_W), **kw)
        self.advantages = torch.zeros((T, N), **kw)
        self.returns = torch.zeros((T, N), **kw)
        self.batch_size = N * T                       # per rank
        self.minibatch_size = self.batch_size // int(cfg.num_minibatches)
        self.params = [p for p in agent.parameters()]
        # one flat gradient bucket; every param.grad is a view of it
        n = sum(p.numel() for p in self.params)
        self.flat_grad = torch.zeros(n, **kw)
        off = 0
        for p in self.params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self.optimizer = torch.optim.Adam(self.params, lr=float(cfg.learning_rate), eps=1e-5,
                                          foreach=self.device.type == "cuda")
        self.next_obs = None
        self.next_done = torch.zeros(N, **kw)
        self.global_step = 0
        self.iteration = 0

    # ------------------------------------------------------------------ rollout
    def reset(self, seed=None):
        obs, _ = self.env.reset(seed=seed)
        self.next_obs = obs.clone()
        self.next_done.zero_()

    @torch.no_grad()
    def rollout_step(self, step: int, env_events=None):
        """One vectorised step of train.py:138-161 (policy sample + env step)."""
        self.obs[step].copy_(self.next_obs)
        self.dones[step].copy_(self.next_done)
        action, logprob, _, value = self.agent.get_action_and_value(self.next_obs, generator=self.gen)
        self.values[step].copy_(value.flatten())
        self.actions[step].copy_(action)
        self.logprobs[step].copy_(logprob)
        if env_events is not None:
            env_events[0].record()
        next_obs, reward, term, trunc, _ = self.env.step(action, info_out=self.infos[step])
        if env_events is not None:
            env_events[1].record()
        self.rewards[step].copy_(reward)
        self.next_obs.copy_(next_obs)
        self.next_done.copy_(term)

    @torch.no_grad()
    def rollout(self):
        """train.py:138-161 for all envs of this rank; no host synchronisation."""
        for step in range(self.T):
            self.rollout_step(step)
        self.global_step += self.N * self.T * self.world

    @torch.no_grad()
    def compute_gae(self):
        """train.py:163-181 via the rt_gae HIP kernel."""
        next_value = self.agent.get_value(self.next_obs).reshape(-1).contiguous()
        if self.gae_fn is not None:
            return self.gae_fn(self, next_value)
        L = _lib.load()
        _lib.check(L.rt_gae(self.T, self.N, self.rewards.data_ptr(), self.values.data_ptr(),
                            self.dones.data_ptr(), next_value.data_ptr(), self.next_done.data_ptr(),
                            float(self.cfg.gamma), float(self.cfg.gae_lambda), self.advantages.data_ptr(),
                            self.returns.data_ptr(), _lib.stream_handle()), "rt_gae")

    # ------------------------------------------------------------------ update
    def _allreduce_(self, t: torch.Tensor, average: bool = True):
        if self.world > 1:
            dist.all_reduce(t)
            if average:
                t.div_(self.world)
        return t

    def _norm_adv(self, adv: torch.Tensor) -> torch.Tensor:
        if self.world == 1:
            return (adv - adv.mean()) / (adv.std() + 1e-8)
        a = adv.double()
        s = torch.stack([a.sum(), (a * a).sum(), torch.tensor(float(a.numel()), dtype=torch.float64,
                                                               device=a.device)])
        self._allreduce_(s, average=False)
        mean = s[0] / s[2]
        var = (s[1] - s[2] * mean * mean) / (s[2] - 1.0)
        return (adv - mean.float()) / (var.clamp_min(0).sqrt().float() + 1e-8)

    def update(self):
        """train.py:183-248."""
        cfg = self.cfg
        b_obs = self.obs.reshape((-1,) + self.obs.shape[2:])
        b_logprobs = self.logprobs.reshape(-1)
        b_actions = self.actions.reshape((-1,) + self.actions.shape[2:])
        b_adv = self.advantages.reshape(-1)
        b_ret = self.returns.reshape(-1)
        b_val = self.values.reshape(-1)
        clip = float(cfg.clip_coef)
        dev = self.device
        clipfrac_sum = torch.zeros((), device=dev)
        n_mb = 0
        for _ in range(int(cfg.update_epochs)):
            perm = torch.randperm(self.batch_size, device=dev, generator=self.gen)
            for start in range(0, self.batch_size, self.minibatch_size):
                mb = perm[start:start + self.minibatch_size]
                _, newlogprob, entropy, newvalue = self.agent.get_action_and_value(b_obs[mb], b_actions[mb])
                logratio = newlogprob - b_logprobs[mb]
                ratio = logratio.exp()
                with torch.no_grad():
                    old_approx_kl = (-logratio).mean()
                    approx_kl = ((ratio - 1) - logratio).mean()
                    clipfrac_sum += ((ratio - 1.0).abs() > clip).float().mean()
                mb_adv = b_adv[mb]
                if cfg.norm_adv:
                    mb_adv = self._norm_adv(mb_adv)
                pg_loss = torch.max(-mb_adv * ratio, -mb_adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
                newvalue = newvalue.view(-1)
                if cfg.clip_vloss:
                    v_unclipped = (newvalue - b_ret[mb]) ** 2
                    v_clipped = b_val[mb] + torch.clamp(newvalue - b_val[mb], -clip, clip)
                    v_loss = 0.5 * torch.max(v_unclipped, (v_clipped - b_ret[mb]) ** 2).mean()
                else:
                    v_loss = 0.5 * ((newvalue - b_ret[mb]) ** 2).mean()
                entropy_loss = entropy.mean()
                loss = pg_loss - float(cfg.ent_coef) * entropy_loss + v_loss * float(cfg.vf_coef)
                self.flat_grad.zero_()
                loss.backward()
                self._allreduce_(self.flat_grad)
                nn.utils.clip_grad_norm_(self.params, float(cfg.max_grad_norm))
                self.optimizer.step()
                n_mb += 1
        self._last = dict(pg_loss=pg_loss.detach(), v_loss=v_loss.detach(), entropy=entropy_loss.detach(),
                          old_approx_kl=old_approx_kl, approx_kl=approx_kl, clipfrac=clipfrac_sum / max(n_mb, 1))
        return n_mb

    # ------------------------------------------------------------------ stats
    @torch.no_grad()
    def iteration_stats(self) -> IterStats:
        """One host sync per iteration: episode statistics of the episodes that
        finished during the rollout (train.py:42-66 logs them per step) and the
        last minibatch's losses (train.py:69-88)."""
        I = self.infos
        done = I[..., 17] > 0.5
        vals = torch.stack([done.sum().double(), (I[..., 18] * done).sum().double(),
                            (I[..., 19] * done).sum().double(), (I[..., 1] * done).sum().double(),
                            (I[..., 2] * done).sum().double(), (I[..., 3] * done).sum().double(),
                            (I[..., 0] * done).sum().double()])
        self._allreduce_(vals, average=False)
        y_pred, y_true = self.values.reshape(-1), self.returns.reshape(-1)
        var_y = y_true.var(unbiased=False)
        ev = torch.where(var_y == 0, torch.tensor(float("nan"), device=y_true.device),
                         1 - (y_true - y_pred).var(unbiased=False) / var_y)
        last = self._last if hasattr(self, "_last") else {}
        host = torch.cat([vals, ev.double().reshape(1)] +
                         [last[k].double().reshape(1) for k in ("pg_loss", "v_loss", "entropy", "old_approx_kl",
                                                                "approx_kl", "clipfrac") if k in last]).cpu().numpy()
        st = IterStats()
        n = int(host[0])
        st.episodes = n
        if n:
            st.episodic_return, st.episodic_length = host[1] / n, host[2] / n
            st.tumour_reward, st.lung_reward, st.distance_reward, st.total_reward = (host[3:7] / n).tolist()
        st.explained_variance = float(host[7])
        if len(host) > 8:
            (st.policy_loss, st.value_loss, st.entropy, st.old_approx_kl, st.approx_kl,
             st.clipfrac) = host[8:14].tolist()
        st.learning_rate = self.optimizer.param_groups[0]["lr"]
        return st

    # ------------------------------------------------------------------ loop
    def anneal(self, iteration: int, num_iterations: int):
        if self.cfg.anneal_lr:
            frac = 1.0 - (iteration - 1.0) / num_iterations
            self.optimizer.param_groups[0]["lr"] = frac * float(self.cfg.learning_rate)

    def train_iteration(self, iteration: int, num_iterations: int) -> IterStats:
        self.anneal(iteration, num_iterations)
        t0 = time.perf_counter()
        self.rollout()
        self.compute_gae()
        torch.cuda.synchronize(self.device)
        t1 = time.perf_counter()
        self.update()
        torch.cuda.synchronize(self.device)
        t2 = time.perf_counter()
        st = self.iteration_stats()
        st.rollout_s, st.update_s = t1 - t0, t2 - t1
        self.iteration = iteration
        return st


def broadcast_parameters(module: nn.Module, src: int = 0):
    """Rank 0's initial weights everywhere (DP replicas start identical)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        for p in module.parameters():
            dist.broadcast(p.data, src)


def explained_variance(y_pred: np.ndarray, y_true: np.ndarray) -> float:
    var_y = np.var(y_true)
    return math.nan if var_y == 0 else float(1 - np.var(y_true - y_pred) / var_y)
