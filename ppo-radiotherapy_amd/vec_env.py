"""Device-resident vectorised environment (the drop-in for the reference's
`gym.vector.SyncVectorEnv([make_env(visionless)] * num_envs)`, train.py:32-39,93-95).

All N envs live in HBM; `step()` is two HIP kernels (include/rtenv.h
rt_env_step) on torch's current stream and never synchronises with the host.
Semantics follow gymnasium 1.0.0:

* NEXT_STEP autoreset: the step after an env terminates ignores its action,
  resets it, and returns the reset observation with reward 0 / terminated
  False; `infos["_reward_components"]` is False for that env (the reference
  env's reset info is `{}`).
* RecordEpisodeStatistics: when an episode ends, `infos["episode"]` holds
  r (sum of step rewards), l (steps), t and the masks `_r/_l/_t`;
  `infos["_episode"]` marks the finishing envs.

`infos` always carries every key (as device tensors with masks) so that no
host sync is needed to build it; `has_episode(infos)` is the sync-on-demand
equivalent of `"episode" in infos` (train.py:160).
"""
from __future__ import annotations

import ctypes
import time

import numpy as np
import torch

from . import _lib, assets, spaces
from .assets import TumourLibrary

# RadiotherapyEnv class constants (environment.py:16-26)
ACTION_SIZE = 6
MAX_TIME_STEPS = 100


def _device_array(x, dtype, device) -> torch.Tensor:
    """A contiguous device tensor of `x` (array-like or tensor, any device)."""
    if torch.is_tensor(x):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device)


class RadiotherapyVecEnv:
    metadata = {"render_modes": ["human"], "render_fps": 30, "autoreset_mode": "NextStep"}

    def __init__(self, num_envs: int, visionless: bool = True, grid=None, device=None, seed: int = 0,
                 library: TumourLibrary | None = None, env_id_base: int = 0, step_mode: str = "dense"):
        """step_mode: "dense" (the reference's full-volume reductions every
        step) or "incremental" (visionless: maintained on the touched voxels;
        same rewards/termination)."""
        if not torch.cuda.is_available():
            raise _lib.RtError("RadiotherapyVecEnv needs a HIP device (MI355X); no CPU fallback")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError("device must be a HIP device")
        self.num_envs = int(num_envs)
        self.visionless = bool(visionless)
        self.library = library if library is not None else assets.library_for(grid or (67, 43, 70))
        self.grid = tuple(self.library.shape)
        self.lung_shape = np.array(self.grid)
        self._seed = int(seed)
        self.single_observation_space = spaces.Box(0.0, 1.0, (9,) if visionless else (4, *self.grid), np.float32)
        self.single_action_space = spaces.Box(-1.0, 1.0, (ACTION_SIZE,), np.float32)
        self.observation_space = spaces.Box(0.0, 1.0, (self.num_envs, *self.single_observation_space.shape), np.float32)
        self.action_space = spaces.Box(-1.0, 1.0, (self.num_envs, ACTION_SIZE), np.float32)

        L = _lib.load()
        cfg = _lib.RtEnvConfig()
        _lib.check(L.rt_env_config_default(cfg), "rt_env_config_default")
        for i in range(3):
            cfg.grid[i] = self.grid[i]
        cfg.num_envs = self.num_envs
        cfg.visionless = 1 if visionless else 0
        self._lungs = np.ascontiguousarray(self.library.lungs.ravel(), dtype=np.uint8)
        self._vox = np.ascontiguousarray(self.library.voxels, dtype=np.int32)
        self._off = np.ascontiguousarray(self.library.offsets, dtype=np.int64)
        cfg.lungs_h = self._lungs.ctypes.data
        cfg.n_tumours = self.library.n_tumours
        cfg.tumour_voxels_h = self._vox.ctypes.data
        cfg.tumour_offsets_h = self._off.ctypes.data
        cfg.seed = self._seed & 0xFFFFFFFFFFFFFFFF
        cfg.env_id_base = int(env_id_base)
        if step_mode not in ("dense", "incremental"):
            raise ValueError("step_mode must be 'dense' or 'incremental'")
        self.step_mode = step_mode if visionless else "dense"
        cfg.step_mode = _lib.STEP_INCREMENTAL if self.step_mode == "incremental" else _lib.STEP_DENSE
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        handle = ctypes_void_p()
        with torch.cuda.device(dev_index):
            _lib.check(L.rt_env_create(cfg, dev_index, handle), "rt_env_create")
        self._h = handle.value
        self._L = L

        N = self.num_envs
        kw = dict(device=self.device)
        self.obs = torch.zeros((N, *self.single_observation_space.shape), dtype=torch.float32, **kw)
        self.reward = torch.zeros(N, dtype=torch.float32, **kw)
        self.terminated = torch.zeros(N, dtype=torch.uint8, **kw)
        self.truncated = torch.zeros(N, dtype=torch.bool, **kw)
        self.info = torch.zeros((N, _lib.INFO_W), dtype=torch.float32, **kw)
        self._episode_start = torch.zeros(N, dtype=torch.float64, **kw)
        self.closed = False

    # ------------------------------------------------------------------ API
    def reset(self, seed: int | None = None, options: dict | None = None):
        """Reset every env (gymnasium VectorEnv.reset).  `options` may hold
        `tumour_ids` (int[N], -1 = sample) and `mask` (bool[N]).  `seed`
        re-keys the tumour-sampling stream (rt_env_reseed): the tumours drawn
        from here on depend only on (seed, global env id)."""
        options = options or {}
        if seed is not None:
            _lib.check(self._L.rt_env_reseed(self._h, int(seed) & 0xFFFFFFFFFFFFFFFF, _lib.stream_handle()),
                       "rt_env_reseed")
            self._seed = int(seed)
        ids = options.get("tumour_ids")
        mask = options.get("mask")
        ids_t = None if ids is None else _device_array(ids, torch.int32, self.device)
        mask_t = None if mask is None else _device_array(mask, torch.uint8, self.device)
        _lib.check(self._L.rt_env_reset(self._h, _lib.ptr(mask_t), _lib.ptr(ids_t), _lib.ptr(self.obs),
                                        _lib.stream_handle()), "rt_env_reset")
        now = time.perf_counter()
        if mask_t is None:
            self._episode_start.fill_(now)
        else:  # RecordEpisodeStatistics' clock restarts for the reset envs only
            self._episode_start = torch.where(mask_t.bool(), now, self._episode_start)
        return self.obs, {}

    def step(self, actions: torch.Tensor, info_out: torch.Tensor | None = None,
             reward_out: torch.Tensor | None = None):
        """`info_out` (f32 [N, INFO_W]) / `reward_out` (f32 [N]), contiguous,
        receive the info rows / rewards instead of the env's own buffers
        (the rollout storage is written in place)."""
        a = actions
        if a.dtype != torch.float32 or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
        if a.shape != (self.num_envs, ACTION_SIZE):
            raise ValueError(f"actions must be [{self.num_envs}, {ACTION_SIZE}], got {tuple(a.shape)}")
        info = self.info if info_out is None else info_out
        if info_out is not None and (info_out.shape != self.info.shape or not info_out.is_contiguous()):
            raise ValueError("info_out must be a contiguous f32 [N, INFO_W] tensor")
        rew = self.reward
        if reward_out is not None:
            if reward_out.shape != (self.num_envs,) or reward_out.dtype != torch.float32 or not reward_out.is_contiguous():
                raise ValueError("reward_out must be a contiguous f32 [N] tensor")
            rew = reward_out
        _lib.check(self._L.rt_env_step(self._h, _lib.ptr(a), _lib.ptr(self.obs), _lib.ptr(rew),
                                       _lib.ptr(self.terminated), _lib.ptr(info), _lib.stream_handle()),
                   "rt_env_step")
        return self.obs, rew, self.terminated.view(torch.bool), self.truncated, self._lazy_infos(info)

    def _lazy_infos(self, info: torch.Tensor) -> "LazyInfos":
        """RecordEpisodeStatistics' wall-clock `t` (gymnasium 1.0: seconds
        since the env's own reset, rounded to 6 decimals): the host time of
        this step minus each env's episode start, which an autoreset on this
        step (info[RT_INFO_STEPPED] = 0) moves to now -- two small device ops
        per facade step, no host sync."""
        now = time.perf_counter()
        ep_t = now - self._episode_start
        self._episode_start = torch.where(info[:, 16] < 0.5, now, self._episode_start)
        return LazyInfos(lambda I: self._infos(I, ep_t), info)

    def step_policy(self, step, info_out: torch.Tensor | None = None, reward_out: torch.Tensor | None = None):
        """Fused rollout step (rt_env_step_policy): the visionless MLP policy
        samples the actions described by `step` (an _lib.RtPolicyStep whose
        pointers name the policy parameters, the observation acted on and the
        rollout-storage slices) and the env steps on them, in one launch per
        step in incremental mode.  Outputs as `step`."""
        if not self.visionless:
            raise ValueError("step_policy: the fused policy is the visionless agent")
        info = self.info if info_out is None else info_out
        rew = self.reward if reward_out is None else reward_out
        _lib.check(self._L.rt_env_step_policy(self._h, ctypes.byref(step), _lib.ptr(self.obs), _lib.ptr(rew),
                                              _lib.ptr(self.terminated), _lib.ptr(info), _lib.stream_handle()),
                   "rt_env_step_policy")
        return self.obs, rew, self.terminated.view(torch.bool), self.truncated, self._lazy_infos(info)

    def rollout_policy(self, rollout) -> int:
        """`rollout.n_steps` fused rollout steps (rt_env_rollout_policy): one
        persistent launch in incremental step mode; in dense mode two env
        groups pipelined over two streams around a persistent k_dense
        (set_rollout_groups(1): the stepwise launches on one stream).  `rollout` is
        an _lib.RtPolicyRollout naming the storage rows of its first step.
        Returns the library's status (RT_ELIMIT: the tumour library is too
        large for the kernel's LDS budget -- step with step_policy instead)."""
        rc = self._L.rt_env_rollout_policy(self._h, ctypes.byref(rollout), _lib.ptr(self.obs),
                                           _lib.ptr(self.terminated), _lib.stream_handle())
        if rc not in (0, _lib.RT_ELIMIT):
            _lib.check(rc, "rt_env_rollout_policy")
        return rc

    def set_rollout_groups(self, groups: int):
        """Env groups of the dense-mode rollout_policy: 2..4 (pipelined streams; default 2) or 1 (the
        stepwise launches on one stream); incremental handles take only 0 (their persistent launch)."""
        _lib.check(self._L.rt_env_set_rollout_groups(self._h, int(groups)), "rt_env_set_rollout_groups")

    def set_next_tumours(self, ids):
        t = torch.as_tensor(np.asarray(ids), dtype=torch.int32, device=self.device)
        _lib.check(self._L.rt_env_set_next_tumours(self._h, _lib.ptr(t), _lib.stream_handle()),
                   "rt_env_set_next_tumours")

    def get_state(self):
        N = self.num_envs
        pose = torch.empty((N, 6), dtype=torch.float64, device=self.device)
        t = torch.empty(N, dtype=torch.int32, device=self.device)
        tum = torch.empty(N, dtype=torch.int32, device=self.device)
        _lib.check(self._L.rt_env_get_state(self._h, _lib.ptr(pose), _lib.ptr(t), _lib.ptr(tum),
                                            _lib.stream_handle()), "rt_env_get_state")
        return pose, t, tum

    def beam_list(self, cap: int | None = None):
        """The beam each env applied on its last step (rt_env_beam_list;
        draw_line.py:4-102 from environment.py:107-110): raw splats in march
        order, (idx i32 [N, cap] C-order flat voxel indices, w f32 [N, cap],
        count i32 [N]); count 0 = the env's last call was its reset."""
        if cap is None:
            cap = 4 * (int(max(self.grid)) + 2)  # <= 4 splats per march iteration
        N = self.num_envs
        idx = torch.zeros((N, cap), dtype=torch.int32, device=self.device)
        w = torch.zeros((N, cap), dtype=torch.float32, device=self.device)
        cnt = torch.zeros(N, dtype=torch.int32, device=self.device)
        _lib.check(self._L.rt_env_beam_list(self._h, int(cap), _lib.ptr(idx), _lib.ptr(w), _lib.ptr(cnt),
                                            _lib.stream_handle()), "rt_env_beam_list")
        return idx, w, cnt

    def set_pose(self, pose: torch.Tensor):
        p = pose.to(device=self.device, dtype=torch.float64).contiguous()
        _lib.check(self._L.rt_env_set_pose(self._h, _lib.ptr(p), _lib.stream_handle()), "rt_env_set_pose")

    def set_tumours(self, ids: torch.Tensor):
        """Current tumour of each env, without a reset (rt_env_set_tumours)."""
        t = ids.to(device=self.device, dtype=torch.int32).contiguous()
        _lib.check(self._L.rt_env_set_tumours(self._h, _lib.ptr(t), _lib.stream_handle()), "rt_env_set_tumours")

    # ---- compact vision rollout storage ----------------------
    def snapshot(self, dose_out: torch.Tensor, pose_out: torch.Tensor, tumour_out: torch.Tensor):
        """Store what the current observation is rendered from: dose f32
        [N, V], pose f64 [N, 6], tumour i32 [N] (4x less than the [N, 4, V]
        vision observation; the lungs, tumour and beam-view channels follow
        from the mask, the tumour id and the pose)."""
        N, V = self.num_envs, int(np.prod(self.grid))
        dose_out.view(N, V).copy_(self.dose().reshape(N, V))
        _lib.check(self._L.rt_env_get_state(self._h, _lib.ptr(pose_out), None, _lib.ptr(tumour_out),
                                            _lib.stream_handle()), "rt_env_get_state")

    def render(self, dose: torch.Tensor, pose: torch.Tensor, tumour: torch.Tensor, rows=None) -> torch.Tensor:
        """Observations [M, 4, D, H, W] of M stored states, bit-identical to
        what the env emitted in them: a render handle is loaded with the states
        and reset with an all-zero mask, which re-emits every observation (the
        same k_dense_vis / k_finish code).  The returned tensor is the render
        handle's buffer, valid until the next render call.  rows: dose is a
        store [R, V] and the states' doses are its rows `rows`, gathered
        straight into the render handle (no intermediate [M, V] copy)."""
        if self.visionless:
            raise ValueError("render() is for vision observations")
        M = int(rows.numel()) if rows is not None else int(dose.shape[0])
        r = getattr(self, "_renderer", None)
        if r is None or r.num_envs < M:
            if r is not None:
                r.close()
            r = RadiotherapyVecEnv(M, visionless=False, library=self.library, device=self.device, seed=self._seed)
            self._renderer = r
            self._render_mask = torch.zeros(M, dtype=torch.uint8, device=self.device)
        V = int(np.prod(self.grid))
        stride = ctypes_int64()
        self._L.rt_env_dose(r._h, stride)
        store = dose.reshape(-1, V) if rows is not None else None
        if (rows is not None and store.is_contiguous() and store.dtype == torch.float32 and V >= stride.value
                and V % 4 == 0 and store.data_ptr() % 16 == 0):
            # the reset below reads the states' doses straight from the store
            ridx = rows.to(torch.int64).contiguous()
            self._render_rows = ridx  # alive until the reset has run
            _lib.check(self._L.rt_env_set_render_source(r._h, _lib.ptr(store), V, _lib.ptr(ridx), M),
                       "rt_env_set_render_source")
        else:
            dst = r.dose().reshape(r.num_envs, V)[:M]
            dst.copy_(store[rows] if rows is not None else dose.reshape(M, V))
        p = torch.zeros((r.num_envs, 6), dtype=torch.float64, device=self.device)
        p[:M] = pose
        p[M:, 4] = 1.0
        t = torch.zeros(r.num_envs, dtype=torch.int32, device=self.device)
        t[:M] = tumour
        _lib.check(self._L.rt_env_set_pose(r._h, _lib.ptr(p), _lib.stream_handle()), "rt_env_set_pose")
        _lib.check(self._L.rt_env_set_tumours(r._h, _lib.ptr(t), _lib.stream_handle()), "rt_env_set_tumours")
        _lib.check(self._L.rt_env_reset(r._h, _lib.ptr(self._render_mask), None, _lib.ptr(r.obs),
                                        _lib.stream_handle()), "rt_env_reset")
        return r.obs[:M]

    def dose(self) -> torch.Tensor:
        """[N, D, H, W] dose volumes: a view of the library-owned rows when
        they are in C order, a C-order copy when the handle keeps them
        lung-first (dense-mode visionless; rt_env_dose_index)."""
        stride = ctypes_int64()
        p = self._L.rt_env_dose(self._h, stride)
        V = int(np.prod(self.grid))
        flat = _tensor_from_ptr(p, (self.num_envs, stride.value), torch.float32, self.device)
        ip = self._L.rt_env_dose_index(self._h)
        if ip:
            pos = _tensor_from_ptr(ip, (V,), torch.int32, self.device).long()
            return flat[:, pos].reshape(self.num_envs, *self.grid)
        return flat[:, :V].reshape(self.num_envs, *self.grid)

    def dose_index(self):
        """i32 [D*H*W] row position of each C-order voxel in the dose rows when
        the handle keeps them lung-first (rt_env_dose_index; a view of
        library memory), else None (C-order rows)."""
        ip = self._L.rt_env_dose_index(self._h)
        if not ip:
            return None
        return _tensor_from_ptr(ip, (int(np.prod(self.grid)),), torch.int32, self.device)

    def kernel_timing(self, capacity: int):
        """Record HIP events around k_beam/k_dense/k_finish for the next
        `capacity` step launches (0 disables); a dense-mode rollout_policy step
        takes one slot per env group."""
        _lib.check(self._L.rt_env_kernel_timing(self._h, int(capacity)), "rt_env_kernel_timing")

    def kernel_timing_read(self):
        """-> ({'k_beam': ms, 'k_dense': ms, 'k_finish': ms} averaged per call, calls)."""
        import ctypes

        ms = (ctypes.c_double * 3)()
        n = ctypes.c_int32()
        _lib.check(self._L.rt_env_kernel_timing_read(self._h, ms, ctypes.byref(n)), "rt_env_kernel_timing_read")
        k = max(n.value, 1)
        return {"k_beam": ms[0] / k, "k_dense": ms[1] / k, "k_finish": ms[2] / k}, n.value

    def close(self):
        r = getattr(self, "_renderer", None)
        if r is not None:
            r.close()
            self._renderer = None
        if getattr(self, "_h", None):
            self._L.rt_env_destroy(self._h)
            self._h = None
        self.closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------------ infos
    def _infos(self, I=None, ep_t=None):
        I = self.info if I is None else I
        stepped = I[:, 16] > 0.5
        ep_done = I[:, 17] > 0.5
        rc = {
            "total": I[:, 0], "tumour": I[:, 1], "lung": I[:, 2], "distance_to_tumour": I[:, 3],
            "_total": stepped, "_tumour": stepped, "_lung": stepped, "_distance_to_tumour": stepped,
        }
        if ep_t is None:
            ep_t = time.perf_counter() - self._episode_start
        ep = {"r": I[:, 18], "l": I[:, 19], "t": torch.where(ep_done, ep_t.round(decimals=6), 0.0),
              "_r": ep_done, "_l": ep_done, "_t": ep_done}
        return {
            "reward_components": rc, "_reward_components": stepped,
            "beam_position": {"translation": I[:, 10:13], "rotation": I[:, 13:16]}, "_beam_position": stepped,
            "doses": {"tumour": I[:, 4], "lung": I[:, 5]}, "_doses": stepped,
            "overshoot": {"translation": I[:, 6:9], "rotation": I[:, 9]}, "_overshoot": stepped,
            "episode": ep, "_episode": ep_done,
        }


class LazyInfos(dict):
    """The gymnasium-style infos dict, built (a few small device ops) only
    when first read -- the rollout loop never reads it."""

    def __init__(self, build, info):
        super().__init__()
        self._build, self._info, self._done = build, info, False

    def _fill(self):
        if not self._done:
            self._done = True
            super().update(self._build(self._info))

    def __getitem__(self, k):
        self._fill()
        return super().__getitem__(k)

    def __contains__(self, k):
        self._fill()
        return super().__contains__(k)

    def __iter__(self):
        self._fill()
        return super().__iter__()

    def __len__(self):
        self._fill()
        return super().__len__()

    def keys(self):
        self._fill()
        return super().keys()

    def items(self):
        self._fill()
        return super().items()

    def values(self):
        self._fill()
        return super().values()

    def get(self, k, default=None):
        self._fill()
        return super().get(k, default)


def has_episode(infos) -> bool:
    """`"episode" in infos` of gymnasium (one device->host sync)."""
    return bool(infos["_episode"].any().item())


# --------------------------------------------------------------------- helpers
def ctypes_void_p():
    import ctypes

    return ctypes.c_void_p()


def ctypes_int64():
    import ctypes

    return ctypes.c_int64()


def _tensor_from_ptr(ptr: int, shape, dtype, device):
    """Non-owning torch view of library-owned device memory."""

    class _Holder:
        def __init__(self, p, nbytes):
            self.__cuda_array_interface__ = {
                "shape": (nbytes // 4,), "typestr": "<f4", "data": (p, False), "version": 3, "strides": None,
            }

    n = int(np.prod(shape))
    t = torch.as_tensor(_Holder(ptr, n * 4), device=device)
    return t.view(dtype).reshape(shape)
