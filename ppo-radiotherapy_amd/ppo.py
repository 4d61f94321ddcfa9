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

import ctypes
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
    # per rollout step with finished episodes (train.py:159-161 logs at each):
    # rows (global_step, n, mean r, mean l, mean tumour, lung, distance, total)
    episode_steps: list = None


def episode_step_sums(infos: torch.Tensor) -> torch.Tensor:
    """[T, 7] per rollout step over the envs whose episode ended there
    (RecordEpisodeStatistics `_r`, info[RT_INFO_EP_DONE]): count, sums of
    episode r and l, and of that final step's reward components tumour, lung,
    distance, total -- what log_episode_statistics averages (train.py:42-66)."""
    I = infos
    done = (I[..., 17] > 0.5).double()
    cols = [I[..., 18], I[..., 19], I[..., 1], I[..., 2], I[..., 3], I[..., 0]]
    return torch.stack([done.sum(1)] + [(c.double() * done).sum(1) for c in cols], 1)


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
        # the collective code path (all-reduces between the update kernels): on
        # exactly when world > 1; tests/test_gpu_rccl.py forces it at world 1 to run
        # the RCCL calls against the single-call update on one GPU
        self.collective = world > 1
        self.gen = generator
        N, T = env.num_envs, int(cfg.num_steps)
        self.N, self.T = N, T
        obs_shape = env.single_observation_space.shape
        act_shape = env.single_action_space.shape
        kw = dict(device=self.device)
        # vision on the HIP env: store (dose, pose, tumour) per step and render
        # observations at update time instead of [T, N, 4, V]
        self.compact_obs = (len(obs_shape) == 4 and hasattr(env, "render") and hasattr(env, "snapshot")
                            and bool(getattr(cfg, "compact_vision_rollout", True)))
        if self.compact_obs:
            V = int(np.prod(obs_shape[1:]))
            self.obs = None
            self.dose_snap = torch.zeros((T, N, V), **kw)
            self.pose_snap = torch.zeros((T, N, 6), dtype=torch.float64, **kw)
            self.tumour_snap = torch.zeros((T, N), dtype=torch.int32, **kw)
        else:
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
        n = sum(p.numel() for p in self.params)
        # fused HIP update (rt_ppo_update: loss + backward + clip + Adam in 3
        # kernels per minibatch) for the visionless 64-wide agent
        self.fused_update = (bool(getattr(cfg, "fused_update", True)) and self.device.type == "cuda"
                             and self._agent_fusable(agent)
                             and self.batch_size % self.minibatch_size == 0)
        if self.fused_update:
            # parameters become views of one flat buffer (Adam runs over it)
            self.flat_param = torch.empty(n, dtype=self.params[0].dtype, **kw)
            off = 0
            with torch.no_grad():
                for p in self.params:
                    k = p.numel()
                    self.flat_param[off:off + k].copy_(p.reshape(-1))
                    p.data = self.flat_param[off:off + k].view_as(p)
                    off += k
            self._exp_avg = torch.zeros_like(self.flat_param)
            self._exp_avg_sq = torch.zeros_like(self.flat_param)
            self._adam_step = 0
            self._ppo_stats = torch.zeros(6, **kw)
            self._ppo_accum = torch.zeros(6, **kw)
            # arithmetic of the fused grad kernel's 64x64 products: "f32" (the
            # reference's) or "bf16x3" (rt_ppo_hparams.precision, per call)
            prec = str(getattr(cfg, "update_precision", "f32"))
            if prec not in _lib.PPO_PREC:
                raise ValueError(f"update_precision {prec!r}: expected one of {sorted(_lib.PPO_PREC)}")
            self._update_prec = _lib.PPO_PREC[prec]
        # arithmetic of the C3D forward products (vision agent): "f32" (the
        # reference's, the default) or "bf16x3"; the extractor passes it per
        # call in each stage's rt_conv_layer
        cprec = str(getattr(cfg, "conv_precision", None) or "f32")
        if cprec not in _lib.CONV_PREC:
            raise ValueError(f"conv_precision {cprec!r}: expected one of {sorted(_lib.CONV_PREC)}")
        self.conv_precision = cprec
        fe = getattr(agent, "features_extractor", None)
        if fe is not None and hasattr(fe, "set_conv_precision"):
            fe.set_conv_precision(cprec)
        # one flat gradient bucket; every param.grad is a view of it
        self.flat_grad = torch.zeros(n, dtype=self.params[0].dtype, **kw)
        off = 0
        for p in self.params:
            p.grad = self.flat_grad[off:off + p.numel()].view_as(p)
            off += p.numel()
        self._last_stats = None
        self._dp_comm = None  # the library's RCCL communicator (_native_dp), built on first use
        self.optimizer = torch.optim.Adam(self.params, lr=float(cfg.learning_rate), eps=1e-5,
                                          foreach=self.device.type == "cuda")
        self.max_minibatches = 0  # >0: stop the update after this many minibatch steps (benchmarks)
        self.record_perms = None  # a list: the fused update appends each epoch's permutation (tests)
        # fused rollout policy step (rt_policy_sample): the visionless 64-wide
        # MLP agent on the HIP env; otherwise the torch path below
        self.fused_policy = (bool(getattr(cfg, "fused_policy", True)) and self.device.type == "cuda"
                             and self._fusable(agent, env))
        # the policy fused into the env step (rt_env_step_policy): one launch per
        # step in incremental mode; same bits as rt_policy_sample + rt_env_step
        self.fused_env_step = (self.fused_policy and bool(getattr(cfg, "fused_env_step", True))
                               and getattr(env, "visionless", False))
        self._step_structs = None
        # ... and whole rollout runs in one call (rt_env_rollout_policy): one
        # persistent launch in incremental step mode, two pipelined env groups
        # in dense mode; same bits as step_policy
        self.fused_rollout = self.fused_env_step and bool(getattr(cfg, "fused_rollout", True))
        self._policy_counter = 0
        self._policy_seed = int(getattr(cfg, "seed", 0)) * 1_000_003 + 7919 * rank + 1
        self._done_valid = False
        if self.fused_policy or self.fused_update:
            import ctypes

            named = dict(agent.named_parameters())
            self._policy_params = [named[k] for k in self.POLICY_ORDER]
            self._policy_ptrs = (ctypes.c_void_p * 13)(*[p.data_ptr() for p in self._policy_params])
        if self.fused_update:
            L = _lib.load()
            self._grad_ptrs = (ctypes.c_void_p * 13)(*[p.grad.data_ptr() for p in self._policy_params])
            self._hp = _lib.RtPpoHparams(
                clip_coef=float(cfg.clip_coef), clip_vloss=int(bool(cfg.clip_vloss)), norm_adv=int(bool(cfg.norm_adv)),
                ent_coef=float(cfg.ent_coef), vf_coef=float(cfg.vf_coef), max_grad_norm=float(cfg.max_grad_norm),
                adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5)
            n_mb = self.batch_size // self.minibatch_size
            E = max(1, int(cfg.update_epochs))
            # rt_ppo_adv_stats (all epochs' minibatches at once) shares the workspace
            self._ws = torch.empty(max(int(L.rt_ppo_workspace_floats(self.minibatch_size)), 128 * n_mb * E), **kw)
            self._norm_ws = torch.empty(256, **kw)
            self._perm_buf = torch.empty((E, self.batch_size), dtype=torch.int64, **kw)  # every epoch's shuffle
            self._adv_stats_buf = torch.empty((E * n_mb, 2), **kw)
            self._adv_sums = torch.empty((E * n_mb, 2), dtype=torch.float64, **kw)
            # epoch shuffle keys: a host generator seeded from the trainer's seed and rank
            self._host_gen = torch.Generator().manual_seed(int(getattr(cfg, "seed", 0)) * 7919 + 104729 * rank + 17)
        self.next_obs = None
        self.next_done = torch.zeros(N, **kw)
        self.global_step = 0
        self.iteration = 0

    # parameter order of the fused kernels (include/rtenv.h rt_policy_sample)
    POLICY_ORDER = ["actor_mean.0.weight", "actor_mean.0.bias", "actor_mean.2.weight", "actor_mean.2.bias",
                    "actor_mean.4.weight", "actor_mean.4.bias", "actor_logstd", "critic.0.weight", "critic.0.bias",
                    "critic.2.weight", "critic.2.bias", "critic.4.weight", "critic.4.bias"]

    @staticmethod
    def _agent_fusable(agent) -> bool:
        from .networks import PPO

        return (isinstance(agent, PPO) and agent.feature_dim == 64
                and tuple(agent.observation_shape) == (9,) and tuple(agent.action_space) == (6,)
                and all(p.dtype == torch.float32 and p.is_contiguous() for p in agent.parameters()))

    @classmethod
    def _fusable(cls, agent, env) -> bool:
        from .vec_env import RadiotherapyVecEnv

        return isinstance(env, RadiotherapyVecEnv) and cls._agent_fusable(agent)

    # ------------------------------------------------------------------ rollout
    def reset(self, seed=None):
        obs, _ = self.env.reset(seed=seed)
        # compact vision storage: the policy reads the env's own obs buffer
        self.next_obs = obs if self.compact_obs else obs.clone()
        self.next_done.zero_()
        self._done_valid = False

    def _rollout_step_fused(self, step: int, env_events=None):
        """train.py:138-158 as two native calls: rt_policy_sample writes
        obs/done/action/logprob/value of this step into the storage, then the
        env steps on storage actions[step] and writes rewards[step]/infos[step]."""
        env = self.env
        if self.fused_env_step and getattr(env, "visionless", False):
            if self._step_structs is None:
                self._step_structs = [_lib.RtPolicyStep(
                    params=ctypes.cast(self._policy_ptrs, ctypes.POINTER(ctypes.c_void_p)), n_params=13,
                    obs_store=self.obs[t].data_ptr(), done_store=self.dones[t].data_ptr(),
                    act_store=self.actions[t].data_ptr(), logp_store=self.logprobs[t].data_ptr(),
                    value_store=self.values[t].data_ptr(), seed=self._policy_seed, env_id_base=self.rank * self.N)
                    for t in range(self.T)]
            st = self._step_structs[step]
            st.obs_in = env.obs.data_ptr()
            st.done_in = env.terminated.data_ptr() if self._done_valid else None
            st.counter = self._policy_counter
            self._policy_counter += 1
            if env_events is not None:
                env_events[0].record()
            env.step_policy(st, info_out=self.infos[step], reward_out=self.rewards[step])
            if env_events is not None:
                env_events[1].record()
            self._done_valid = True
            return
        L = _lib.load()
        stream = _lib.stream_handle()
        _lib.check(L.rt_policy_sample(self._policy_ptrs, 13, self.N, env.obs.data_ptr(),
                                      env.terminated.data_ptr() if self._done_valid else None,
                                      self.obs[step].data_ptr(), self.dones[step].data_ptr(),
                                      self.actions[step].data_ptr(), self.logprobs[step].data_ptr(),
                                      self.values[step].data_ptr(), self._policy_seed, self._policy_counter,
                                      self.rank * self.N, stream), "rt_policy_sample")
        self._policy_counter += 1
        if env_events is not None:
            env_events[0].record()
        env.step(self.actions[step], info_out=self.infos[step], reward_out=self.rewards[step])
        if env_events is not None:
            env_events[1].record()
        self._done_valid = True

    @torch.no_grad()
    def rollout_step(self, step: int, env_events=None):
        """One vectorised step of train.py:138-161 (policy sample + env step)."""
        if self.fused_policy:
            return self._rollout_step_fused(step, env_events)
        if self.compact_obs:
            self.env.snapshot(self.dose_snap[step], self.pose_snap[step], self.tumour_snap[step])
        else:
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
        if not self.compact_obs:
            self.next_obs.copy_(next_obs)
        self.next_done.copy_(term)

    @torch.no_grad()
    def rollout(self):
        """train.py:138-161 for all envs of this rank; no host synchronisation."""
        self.rollout_steps(0, self.T)
        self.global_step += self.N * self.T * self.world

    @torch.no_grad()
    def rollout_steps(self, first: int, count: int):
        """Rollout steps first .. first+count-1 (storage rows): one library
        call when the env supports it (rt_env_rollout_policy), otherwise step
        by step."""
        if not (self.fused_rollout and getattr(self.env, "visionless", False)):
            for step in range(first, first + count):
                self.rollout_step(step)
            return
        if self.env.rollout_policy(self._rollout_struct(first, count)) == _lib.RT_ELIMIT:
            self.fused_rollout = False  # library too large for the persistent kernel's LDS
            return self.rollout_steps(first, count)
        self._policy_counter += count
        self._done_valid = True

    @staticmethod
    def _row_ptr(t: torch.Tensor, row: int) -> int:
        """Device address of t[row] without building the view (a CUDA view op
        runs a device guard: two HIP calls each, on the host's critical path
        between a synchronise and the rollout call's first launch)."""
        return t.data_ptr() + row * t.stride(0) * t.element_size()

    def _storage_rows(self, first: int):
        """The storage rows' addresses of a rollout call starting at row
        `first` (obs, dones, actions, logprobs, values, rewards, infos), cached
        per `first`: the storage is allocated once, and Tensor.stride alone
        costs ~2 us of argument parsing -- 20-35 us of host time per call
        before its first launch, inside every timed window."""
        cache = self.__dict__.setdefault("_rows_cache", {})
        hit = cache.get(first)
        if hit is None or hit[0] != self.actions.data_ptr():
            rp = self._row_ptr
            hit = cache[first] = (self.actions.data_ptr(),
                                  tuple(rp(t, first) for t in (self.obs, self.dones, self.actions, self.logprobs,
                                                               self.values, self.rewards, self.infos)))
        return hit[1]

    def _rollout_struct(self, first: int, count: int):
        """rt_policy_rollout for storage rows first .. first+count-1 (one
        cached struct, refilled: the call's host time before its first launch
        is part of every timed window)."""
        env = self.env
        ro = getattr(self, "_ro_cache", None)
        if ro is None:
            ro = self._ro_cache = _lib.RtPolicyRollout()
            ro.step.params = ctypes.cast(self._policy_ptrs, ctypes.POINTER(ctypes.c_void_p))
            ro.step.n_params = 13
        st = ro.step
        key = (first, count, self._done_valid, self._policy_seed, env.obs.data_ptr())
        if getattr(self, "_ro_key", None) == key:  # the usual call: only the Philox counter moved
            st.counter = self._policy_counter
            return ro
        self._ro_key = key
        obs_r, done_r, act_r, logp_r, value_r, rew_r, info_r = self._storage_rows(first)
        st.obs_in = env.obs.data_ptr()
        st.done_in = env.terminated.data_ptr() if self._done_valid else None
        st.obs_store = obs_r
        st.done_store = done_r
        st.act_store = act_r
        st.logp_store = logp_r
        st.value_store = value_r
        st.seed = self._policy_seed
        st.counter = self._policy_counter
        st.env_id_base = self.rank * self.N
        ro.n_steps = count
        ro.reward_store = rew_r
        ro.info_store = info_r
        return ro

    def _sync_next(self):
        """Fused rollout keeps next_obs/next_done in the env's buffers."""
        if self.fused_policy:
            self.next_obs.copy_(self.env.obs)
            if self._done_valid:
                self.next_done.copy_(self.env.terminated)

    @torch.no_grad()
    def compute_gae(self):
        """train.py:163-181 via the rt_gae HIP kernel."""
        self._sync_next()
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
        if self.collective:
            dist.all_reduce(t)
            if average:
                t.div_(self.world)
        return t

    def _adv_stats(self, adv: torch.Tensor):
        """(mean, unbiased std) of a minibatch's advantages (train.py:215-218).
        World 1: torch's own f32 statistics, as the reference.  Collective: the
        statistics of the UNION of the ranks' minibatches (the single-process
        minibatch the DP update stands for), from one f64 all-reduce of
        [sum, sum of squares, count]."""
        if not self.collective:
            return adv.mean(), adv.std()
        a = adv.double()
        s = torch.stack([a.sum(), (a * a).sum(), torch.tensor(float(a.numel()), dtype=torch.float64,
                                                               device=a.device)])
        self._allreduce_(s, average=False)
        mean = s[0] / s[2]
        var = (s[1] - s[2] * mean * mean) / (s[2] - 1.0)
        return mean.float(), var.clamp_min(0).sqrt().float()

    def _norm_adv(self, adv: torch.Tensor) -> torch.Tensor:
        mean, std = self._adv_stats(adv)
        return (adv - mean) / (std + 1e-8)

    def _minibatch_loss_backward(self, mb, adv_mean=None, adv_std=None):
        """train.py:200-246 for one minibatch: losses, then backward into the
        flat gradient bucket.  Returns the logged statistics.  With
        cfg.micro_batch set (vision: C3D activations of a whole minibatch do not
        fit), the minibatch is processed in slices whose gradients accumulate;
        each slice's loss is weighted by its share, so the gradient equals the
        full-minibatch one.  The advantage statistics are taken once, before
        the slices, over the whole minibatch -- over the union of the ranks'
        minibatches when the update is collective (_adv_stats)."""
        micro = int(getattr(self.cfg, "micro_batch", 0) or 0)
        if micro and mb.numel() > micro:
            if self.cfg.norm_adv and adv_mean is None:
                adv_mean, adv_std = self._adv_stats(self._b_adv[mb])
            self.flat_grad.zero_()
            acc = None
            n = mb.numel()
            for s in range(0, n, micro):
                part = mb[s:s + micro]
                st = self._loss_backward(part, adv_mean, adv_std, weight=part.numel() / n, zero=False)
                acc = st * (part.numel() / n) if acc is None else acc + st * (part.numel() / n)
            return acc
        return self._loss_backward(mb, adv_mean, adv_std)

    def _obs_rows(self, mb):
        """Observations of the batch rows mb (rendered from the stored states
        in compact vision mode)."""
        if not self.compact_obs:
            return self._b_obs[mb]
        return self.env.render(self._b_dose, self._b_pose[mb], self._b_tumour[mb], rows=mb)

    def _loss_backward(self, mb, adv_mean=None, adv_std=None, weight: float = 1.0, zero: bool = True):
        cfg = self.cfg
        clip = float(cfg.clip_coef)
        _, newlogprob, entropy, newvalue = self.agent.get_action_and_value(self._obs_rows(mb), self._b_actions[mb])
        logratio = newlogprob - self._b_logprobs[mb]
        ratio = logratio.exp()
        with torch.no_grad():
            old_approx_kl = (-logratio).mean()
            approx_kl = ((ratio - 1) - logratio).mean()
            clipfrac = ((ratio - 1.0).abs() > clip).float().mean()
        mb_adv = self._b_adv[mb]
        if cfg.norm_adv:
            if adv_mean is None:
                mb_adv = self._norm_adv(mb_adv)
            else:
                mb_adv = (mb_adv - adv_mean) / (adv_std + 1e-8)
        pg_loss = torch.max(-mb_adv * ratio, -mb_adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
        newvalue = newvalue.view(-1)
        b_ret, b_val = self._b_ret[mb], self._b_val[mb]
        if cfg.clip_vloss:
            v_unclipped = (newvalue - b_ret) ** 2
            v_clipped = b_val + torch.clamp(newvalue - b_val, -clip, clip)
            v_loss = 0.5 * torch.max(v_unclipped, (v_clipped - b_ret) ** 2).mean()
        else:
            v_loss = 0.5 * ((newvalue - b_ret) ** 2).mean()
        entropy_loss = entropy.mean()
        loss = pg_loss - float(cfg.ent_coef) * entropy_loss + v_loss * float(cfg.vf_coef)
        if zero:
            self.flat_grad.zero_()
        (loss * weight if weight != 1.0 else loss).backward()
        return torch.stack([pg_loss.detach(), v_loss.detach(), entropy_loss.detach(), old_approx_kl,
                            approx_kl, clipfrac])

    def _optimizer_step(self, grad_div: int = 1):
        """clip_grad_norm_ + Adam (train.py:244-246).  grad_div > 1: the flat
        bucket holds the ranks' SUM (all-reduced, not yet averaged); the
        average and the clip are one multiply by min(1, max_norm / (||g|| /
        world + 1e-6)) / world -- torch's clip coefficient of the averaged
        gradient, without a division pass over the bucket of its own."""
        max_norm = float(self.cfg.max_grad_norm)
        if grad_div == 1:
            nn.utils.clip_grad_norm_(self.params, max_norm)
        else:
            norm = torch.linalg.vector_norm(self.flat_grad) / grad_div
            coef = (max_norm / (norm + 1e-6)).clamp(max=1.0)
            self.flat_grad.mul_(coef / grad_div)
        self.optimizer.step()

    def _bind_batch(self):
        if self.compact_obs:
            self._b_obs = None
            self._b_dose = self.dose_snap.view(-1, self.dose_snap.shape[-1])
            self._b_pose = self.pose_snap.view(-1, 6)
            self._b_tumour = self.tumour_snap.view(-1)
        else:
            self._b_obs = self.obs.reshape((-1,) + self.obs.shape[2:])
        self._b_logprobs = self.logprobs.reshape(-1)
        self._b_actions = self.actions.reshape((-1,) + self.actions.shape[2:])
        self._b_adv = self.advantages.reshape(-1)
        self._b_ret = self.returns.reshape(-1)
        self._b_val = self.values.reshape(-1)

    def _batch_struct(self):
        return _lib.RtPpoBatch(self._b_obs.data_ptr(), self._b_actions.data_ptr(), self._b_logprobs.data_ptr(),
                               self._b_adv.data_ptr(), self._b_ret.data_ptr(), self._b_val.data_ptr(),
                               self.batch_size)

    def _epochs_perm_stats(self, L, stream, n_mb: int, epochs: int):
        """The shuffles of `epochs` epochs (rt_ppo_shuffle_epochs, one key per
        epoch drawn in order from the trainer's generator, so epoch e has the
        permutation a per-epoch draw would give) and the advantage statistics
        of all their minibatches (rt_ppo_adv_stats; with world > 1 the sums are
        all-reduced, once for all epochs) -- three launches per update instead
        of three per epoch."""
        keys = (ctypes.c_uint64 * epochs)(*[int(torch.randint(0, 2 ** 62, (1,), generator=self._host_gen).item())
                                            for _ in range(epochs)])
        perm = self._perm_buf[:epochs]
        if not self.cfg.norm_adv:
            _lib.check(L.rt_ppo_shuffle_epochs(self.batch_size, epochs, keys, perm.data_ptr(), stream),
                       "rt_ppo_shuffle_epochs")
            stats = None
        else:
            # the shuffles and the minibatch statistics in one pass (rt_ppo_shuffle_adv)
            k = epochs * n_mb
            stats = self._adv_stats_buf[:k]
            sums = self._adv_sums[:k] if self.collective else None
            _lib.check(L.rt_ppo_shuffle_adv(self.batch_size, epochs, keys, perm.data_ptr(), self._b_adv.data_ptr(),
                                            self.minibatch_size, _lib.ptr(sums),
                                            None if self.collective else stats.data_ptr(), self._ws.data_ptr(),
                                            self._ws.numel(), stream), "rt_ppo_shuffle_adv")
            if self.collective:
                # this rank's (sum, sum of squares) per minibatch -> ONE all-reduce
                # of [k, 2] f64 -> global (mean, std) over mbs x world rows
                dist.all_reduce(sums)
                _lib.check(L.rt_ppo_adv_finalize(sums.data_ptr(), self.minibatch_size * self.world, k,
                                                 stats.data_ptr(), stream), "rt_ppo_adv_finalize")
        if self.record_perms is not None:  # test hook: the epochs' minibatch rows
            self.record_perms.extend(p.clone() for p in perm)
        return perm, stats

    def _native_dp(self):
        """The library's own RCCL communicator for the data-parallel fused
        update (rt_ppo_update_dp), built once over the torch.distributed group:
        rank 0 draws the id, a broadcast hands it to every rank.  None -- the
        per-minibatch loop of rt_ppo_grad / torch.distributed.all_reduce /
        rt_adam_step -- on gloo groups (the CPU and same-device rehearsals) or
        with cfg.native_dp = False."""
        if self._dp_comm is None:
            self._dp_comm = False
            if (bool(getattr(self.cfg, "native_dp", True)) and self.device.type == "cuda" and dist.is_available()
                    and dist.is_initialized() and dist.get_backend() == "nccl"):
                L = _lib.load()
                ident = (ctypes.c_uint8 * _lib.DP_ID_BYTES)()
                if dist.get_rank() == 0:
                    _lib.check(L.rt_dp_unique_id(ident), "rt_dp_unique_id")
                t = torch.tensor(list(bytes(ident)), dtype=torch.uint8, device=self.device)
                dist.broadcast(t, 0)
                ident = (ctypes.c_uint8 * _lib.DP_ID_BYTES)(*t.cpu().tolist())
                h = ctypes.c_void_p()
                _lib.check(L.rt_dp_comm_create(ident, dist.get_world_size(), dist.get_rank(),
                                               self.device.index or 0, ctypes.byref(h)), "rt_dp_comm_create")
                self._dp_comm = h
        return self._dp_comm or None

    def _update_fused(self):
        """train.py:183-248 through the fused kernels: every epoch's shuffle and
        (all-reduced) minibatch advantage statistics up front, then per
        minibatch rt_ppo_grad + the clip/Adam step (world 1: all of it is ONE
        rt_ppo_update call; world > 1 over RCCL: ONE rt_ppo_update_dp call, the
        library all-reducing the flat gradient bucket between the grad and Adam
        kernels; over gloo: a Python loop around torch.distributed.all_reduce)."""
        self._bind_batch()
        L = _lib.load()
        self._hp.precision = self._update_prec  # per call (rt_ppo_hparams.precision)
        stream = _lib.stream_handle()
        batch = self._batch_struct()
        hp = ctypes.byref(self._hp)
        mbs = self.minibatch_size
        n_mb = self.batch_size // mbs
        lr = float(self.optimizer.param_groups[0]["lr"])
        n = self.flat_param.numel()
        self._ppo_accum.zero_()
        total = int(self.cfg.update_epochs) * n_mb
        if self.max_minibatches:
            total = min(total, self.max_minibatches)
        epochs = -(-total // n_mb)
        if total < 1:
            return 0
        perm, adv = self._epochs_perm_stats(L, stream, n_mb, epochs)
        if not self.collective:
            _lib.check(L.rt_ppo_update(self._policy_ptrs, self._grad_ptrs, ctypes.byref(batch), perm.data_ptr(),
                                       mbs, total, _lib.ptr(adv), hp, self.flat_param.data_ptr(),
                                       self.flat_grad.data_ptr(), self._exp_avg.data_ptr(),
                                       self._exp_avg_sq.data_ptr(), n, self._adam_step + 1, lr,
                                       self._ws.data_ptr(), self._ws.numel(), self._ppo_stats.data_ptr(),
                                       self._ppo_accum.data_ptr(), stream), "rt_ppo_update")
            self._adam_step += total
        elif self._native_dp() is not None:
            # the whole data-parallel update in one call: grad, RCCL SUM all-reduce
            # of the flat gradient, clip + Adam (grad_div = world) per minibatch
            _lib.check(L.rt_ppo_update_dp(self._policy_ptrs, self._grad_ptrs, ctypes.byref(batch), perm.data_ptr(),
                                          mbs, total, _lib.ptr(adv), hp, self.flat_param.data_ptr(),
                                          self.flat_grad.data_ptr(), self._exp_avg.data_ptr(),
                                          self._exp_avg_sq.data_ptr(), n, self._adam_step + 1, lr,
                                          self._ws.data_ptr(), self._ws.numel(), self._ppo_stats.data_ptr(),
                                          self._ppo_accum.data_ptr(), self._dp_comm, stream), "rt_ppo_update_dp")
            self._adam_step += total
        else:
            for i in range(total):
                _lib.check(L.rt_ppo_grad(self._policy_ptrs, self._grad_ptrs, ctypes.byref(batch),
                                         perm.data_ptr() + 8 * i * mbs, mbs,
                                         None if adv is None else adv.data_ptr() + 8 * i, hp,
                                         self._ws.data_ptr(), self._ws.numel(), self._ppo_stats.data_ptr(),
                                         self._ppo_accum.data_ptr(), stream), "rt_ppo_grad")
                # SUM all-reduce; rt_adam_step divides by the world size itself
                # (grad.div_(world) without a kernel of its own)
                self._allreduce_(self.flat_grad, average=False)
                self._adam_step += 1
                _lib.check(L.rt_adam_step(n, self.flat_param.data_ptr(), self.flat_grad.data_ptr(),
                                          self._exp_avg.data_ptr(), self._exp_avg_sq.data_ptr(),
                                          self._adam_step, lr, hp, self.world, self._norm_ws.data_ptr(),
                                          stream), "rt_adam_step")
        self._last_stats = torch.cat([self._ppo_stats[:5], (self._ppo_accum[5] / total).reshape(1)])
        return total

    def update(self):
        """train.py:183-248: update_epochs x num_minibatches optimizer steps."""
        if self.fused_update:
            return self._update_fused()
        self._bind_batch()
        dev = self.device
        stats_sum = torch.zeros(6, device=dev)
        n_mb = 0
        for _ in range(int(self.cfg.update_epochs)):
            perm = torch.randperm(self.batch_size, device=dev, generator=self.gen)
            if self.record_perms is not None:  # test hook: the epochs' minibatch rows
                self.record_perms.append(perm.clone())
            for start in range(0, self.batch_size, self.minibatch_size):
                mb = perm[start:start + self.minibatch_size]
                st = self._minibatch_loss_backward(mb)
                stats_sum[5] += st[5]
                self._allreduce_(self.flat_grad, average=False)  # SUM; averaged inside the clip multiply
                self._optimizer_step(self.world if self.collective else 1)
                n_mb += 1
                if self.max_minibatches and n_mb >= self.max_minibatches:
                    break
            if self.max_minibatches and n_mb >= self.max_minibatches:
                break
        self._last_stats = torch.cat([st[:5], (stats_sum[5] / max(n_mb, 1)).reshape(1)])
        return n_mb

    # ------------------------------------------------------------------ stats
    @torch.no_grad()
    def iteration_stats(self) -> IterStats:
        """One host sync per iteration: episode statistics of the episodes that
        finished during the rollout (train.py:42-66 logs them per step) and the
        last minibatch's losses (train.py:69-88)."""
        per_step = episode_step_sums(self.infos)       # [T, 7]
        self._allreduce_(per_step, average=False)     # global over ranks, per step
        vals = per_step.sum(0)
        y_pred, y_true = self.values.reshape(-1), self.returns.reshape(-1)
        var_y = y_true.var(unbiased=False)
        ev = torch.where(var_y == 0, torch.tensor(float("nan"), device=y_true.device),
                         1 - (y_true - y_pred).var(unbiased=False) / var_y)
        parts = [vals, ev.double().reshape(1)]
        if getattr(self, "_last_stats", None) is not None:
            # losses / KL / clipfrac of this rank's minibatches: averaged over
            # the ranks, so the logged scalars are global like the episode stats
            parts.append(self._allreduce_(self._last_stats.double().clone()))
        parts.append(per_step.reshape(-1))
        host = torch.cat(parts).cpu().numpy()
        steps = host[-per_step.numel():].reshape(per_step.shape)
        host = host[:-per_step.numel()]
        st = IterStats()
        # the rollout's steps end at global_step; step t of it at gs0 + (t + 1) N_global
        n_global = self.N * self.world
        gs0 = self.global_step - self.T * n_global
        st.episode_steps = [(gs0 + (t + 1) * n_global, int(r[0]), *(r[1:] / r[0]).tolist())
                            for t, r in enumerate(steps) if r[0] > 0]
        n = int(host[0])
        st.episodes = n
        if n:
            st.episodic_return, st.episodic_length = host[1] / n, host[2] / n
            st.tumour_reward, st.lung_reward, st.distance_reward, st.total_reward = (host[3:7] / n).tolist()
        st.explained_variance = float(host[7])
        if len(host) > 8:
            (st.policy_loss, st.value_loss, st.entropy, st.old_approx_kl, st.approx_kl,
             st.clipfrac) = host[8:14].tolist()
        st.learning_rate = float(self.optimizer.param_groups[0]["lr"])
        return st

    # ------------------------------------------------------------------ loop
    def anneal(self, iteration: int, num_iterations: int):
        if self.cfg.anneal_lr:
            frac = 1.0 - (iteration - 1.0) / num_iterations
            self.optimizer.param_groups[0]["lr"] = frac * float(self.cfg.learning_rate)

    # ------------------------------------------------------------------ checkpoint / resume
    def check_device_status(self):
        """Raise if a fused update on this device lost the grid arrival of its
        reduce + Adam launch (rt_ppo_status, after the stream sync): the
        parameters are then the last complete minibatch's, and a checkpoint of
        them must not be saved as if the update had run."""
        if self.fused_update:
            torch.cuda.synchronize(self.device)
            _lib.check(_lib.load().rt_ppo_status(), "rt_ppo_status")

    def _rng_states(self) -> dict:
        d = {}
        if self.gen is not None:
            d["gen"] = self.gen.get_state()
        if self.fused_update:
            d["host_gen"] = self._host_gen.get_state()
        return d

    def _reseed_rngs(self, iteration: int):
        """Per-rank sampling/shuffle streams derived from (seed, rank,
        iteration): a resume whose checkpoint has no state for this rank."""
        base = (int(getattr(self.cfg, "seed", 0)) * 1_000_003 + 7919 * self.rank + 104_729 * iteration) & (2 ** 63 - 1)
        if self.gen is not None:
            self.gen.manual_seed(base)
        if self.fused_update:
            self._host_gen.manual_seed(base ^ 0x5DEECE66D)

    def state_dict(self) -> dict:
        """What a resumed run continues from (the reference saves
        the agent's state_dict only, train.py:270-279): agent, optimizer
        (torch Adam state and, for the fused update, the flat Adam moments and
        step count), iteration, global step, the rollout policy's Philox
        counter and EVERY rank's sampling/shuffle generator states (`rng`,
        indexed by rank).  With world > 1 this is a collective (all ranks call
        it; rank 0 writes the file).  The envs are not part of it: a resumed
        run starts fresh episodes on a re-keyed tumour stream (train.py)."""
        d = {"agent": self.agent.state_dict(), "optimizer": self.optimizer.state_dict(),
             "iteration": self.iteration, "global_step": self.global_step, "policy_counter": self._policy_counter,
             "world": self.world}
        mine = self._rng_states()
        if self.world > 1 and dist.is_available() and dist.is_initialized():
            ranks = [None] * self.world
            dist.all_gather_object(ranks, mine)
        else:
            ranks = [mine]
        d["rng"] = ranks
        if self.fused_update:
            d["adam"] = {"exp_avg": self._exp_avg.detach().clone(), "exp_avg_sq": self._exp_avg_sq.detach().clone(),
                         "step": self._adam_step}
        return d

    def load_state_dict(self, d: dict):
        """Inverse of state_dict (parameters are copied in place, so the flat
        parameter / gradient buffers of the fused update keep their views).
        Each rank takes its own generator states; when the checkpoint holds
        none for this rank (another world size) they are re-derived from
        (seed, rank, iteration) so replicas keep distinct streams."""
        with torch.no_grad():
            self.agent.load_state_dict(d["agent"])
        self.optimizer.load_state_dict(d["optimizer"])
        self.iteration = int(d["iteration"])
        self.global_step = int(d["global_step"])
        self._policy_counter = int(d["policy_counter"])
        if self.fused_update:
            a = d.get("adam")
            if a is None:
                raise ValueError("checkpoint has no fused-update Adam state")
            self._exp_avg.copy_(a["exp_avg"])
            self._exp_avg_sq.copy_(a["exp_avg_sq"])
            self._adam_step = int(a["step"])
        rng = d.get("rng")
        if rng is None and ("gen" in d or "host_gen" in d) and self.world == 1 and int(d.get("world", 1)) == 1:
            # checkpoints written before the per-rank list kept the (single)
            # rank's states at the top level: continue them
            rng = [{k: d[k] for k in ("gen", "host_gen") if k in d}]
        if rng is not None and len(rng) == self.world:
            mine = rng[self.rank]
            if self.gen is not None and "gen" in mine:
                self.gen.set_state(mine["gen"].cpu())
            if self.fused_update and "host_gen" in mine:
                self._host_gen.set_state(mine["host_gen"].cpu())
        else:
            import warnings

            warnings.warn(f"checkpoint holds no sampling/shuffle generator state for rank {self.rank} of "
                          f"world {self.world}: streams re-derived from (seed, rank, iteration)")
            self._reseed_rngs(self.iteration)

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
