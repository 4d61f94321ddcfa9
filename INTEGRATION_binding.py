"""rtenv_binding -- the reference-side ctypes binding of librtenv.so.

This is the file INTEGRATION.md §2 describes: a maintainer of the reference
(rmaguado/ppo-radiotherapy) drops it next to train.py and replaces
`gym.vector.SyncVectorEnv([make_env(...)])` (train.py:93-95) and the
`envs.reset` / `envs.step` calls of the rollout (train.py:123, 151-158) with
`GpuVecEnv`.  It is self-contained on purpose (ctypes + numpy + torch only,
no import of this repo's Python package), so it is exactly what the
reference would carry; tests/test_gpu_binding.py imports it and drives it
against the C oracle.

The ABI is include/rtenv.h.  Structs are declared here by hand, as a foreign
binding has to: `rt_env_config.struct_size` (its first member) carries this
declaration's size, and the library rejects a config whose size differs from
its own (RT_EINVAL) instead of reading or writing past it, so a stale copy of
this file fails loudly.  `RTENV_ABI_VERSION` is checked at load.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch  # before the library: torch ships the process's libamdhip64

RTENV_ABI_VERSION = 5
RT_INFO_W = 20  # info row: RT_INFO_* in rtenv.h (0..3 reward_components, 17..19 episode _r / r / l)
RT_STEP_DENSE, RT_STEP_INCREMENTAL = 0, 1

_DEFAULT_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ppo-radiotherapy_amd", "librtenv.so")


class RtEnvConfig(ctypes.Structure):
    """rt_env_config (include/rtenv.h)."""
    _fields_ = [("struct_size", ctypes.c_uint32),
                ("grid", ctypes.c_int32 * 3), ("num_envs", ctypes.c_int32), ("visionless", ctypes.c_int32),
                ("max_time_steps", ctypes.c_int32), ("beam_dose", ctypes.c_float),
                ("lung_dose_threshold", ctypes.c_float), ("tumour_dose_threshold", ctypes.c_float),
                ("min_angle_z", ctypes.c_double), ("movement_speed", ctypes.c_double),
                ("rotation_speed", ctypes.c_float), ("lung_dose_reward", ctypes.c_double),
                ("tumour_dose_reward", ctypes.c_float), ("distance_reward", ctypes.c_double),
                ("lungs_h", ctypes.c_void_p), ("n_tumours", ctypes.c_int32),
                ("tumour_voxels_h", ctypes.c_void_p), ("tumour_offsets_h", ctypes.c_void_p),
                ("seed", ctypes.c_uint64), ("env_id_base", ctypes.c_int64), ("step_mode", ctypes.c_int32)]


_L = None


def load(path: str | None = None):
    """dlopen librtenv.so (after `import torch`) and declare the calls used here."""
    global _L
    if _L is not None:
        return _L
    L = ctypes.CDLL(path or os.environ.get("RT_LIB_PATH", _DEFAULT_LIB))
    vp, P = ctypes.c_void_p, ctypes.POINTER
    L.rt_abi_version.restype = ctypes.c_int
    L.rt_last_error.restype = ctypes.c_char_p
    L.rt_env_config_default.argtypes = [P(RtEnvConfig)]
    L.rt_env_create.argtypes = [P(RtEnvConfig), ctypes.c_int, P(vp)]
    L.rt_env_destroy.argtypes = [vp]
    L.rt_env_destroy.restype = None
    L.rt_env_reset.argtypes = [vp] * 5
    L.rt_env_step.argtypes = [vp] * 7
    for name in ("rt_env_config_default", "rt_env_create", "rt_env_reset", "rt_env_step"):
        getattr(L, name).restype = ctypes.c_int
    if L.rt_abi_version() != RTENV_ABI_VERSION:
        raise RuntimeError(f"librtenv.so ABI {L.rt_abi_version()} != binding ABI {RTENV_ABI_VERSION}")
    _L = L
    return L


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {load().rt_last_error().decode(errors='replace')}")


def tumour_voxels_from_volumes(volumes) -> list[np.ndarray]:
    """The reference keeps each tumour as a dense {0,1} volume on disk
    (environment.py:95 `np.load(f"./data/tumours/{name}")`); the library takes
    sorted flat C-order voxel lists."""
    return [np.flatnonzero(np.asarray(v).ravel() == 1.0).astype(np.int32) for v in volumes]


class GpuVecEnv:
    """N RadiotherapyEnv instances (environment.py:15-273) + SyncVectorEnv
    NEXT_STEP autoreset + RecordEpisodeStatistics, resident on one GPU.

    lungs: RadiotherapyEnv.LUNGS_ARRAY (environment.py:28-30); tumours: voxel
    lists (tumour_voxels_from_volumes).  Tensors live on the current device;
    every call is asynchronous on torch's current stream."""

    def __init__(self, num_envs: int, lungs: np.ndarray, tumours, seed: int = 0, env_id_base: int = 0,
                 incremental: bool = False):
        L = load()
        cfg = RtEnvConfig()
        cfg.struct_size = ctypes.sizeof(RtEnvConfig)
        _check(L.rt_env_config_default(ctypes.byref(cfg)), "rt_env_config_default")
        cfg.grid[:] = [int(s) for s in lungs.shape]
        cfg.num_envs = int(num_envs)
        self._keep = (np.ascontiguousarray(lungs, np.uint8).ravel(), np.concatenate(tumours).astype(np.int32),
                      np.concatenate([[0], np.cumsum([len(t) for t in tumours])]).astype(np.int64))
        cfg.lungs_h, cfg.tumour_voxels_h, cfg.tumour_offsets_h = (a.ctypes.data for a in self._keep)
        cfg.n_tumours = len(tumours)
        cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        cfg.env_id_base = int(env_id_base)
        cfg.step_mode = RT_STEP_INCREMENTAL if incremental else RT_STEP_DENSE
        self.device = torch.device("cuda", torch.cuda.current_device())
        h = ctypes.c_void_p()
        _check(L.rt_env_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)), "rt_env_create")
        self._h = h
        self.num_envs = int(num_envs)
        kw = dict(device=self.device)
        self.obs = torch.zeros((self.num_envs, 9), **kw)
        self.reward = torch.zeros(self.num_envs, **kw)
        self.terminated = torch.zeros(self.num_envs, dtype=torch.uint8, **kw)
        self.info = torch.zeros((self.num_envs, RT_INFO_W), **kw)

    @staticmethod
    def _stream():
        return torch.cuda.current_stream().cuda_stream or None

    def reset(self, tumour_ids=None):
        """envs.reset (train.py:123); tumour_ids (int[N], -1 = sample) pins the
        np.random.choice draw of environment.py:90."""
        ids = None if tumour_ids is None else torch.as_tensor(np.asarray(tumour_ids, np.int32), device=self.device)
        _check(load().rt_env_reset(self._h, None, None if ids is None else ids.data_ptr(), self.obs.data_ptr(),
                                   self._stream()), "rt_env_reset")
        return self.obs

    def step(self, actions: torch.Tensor):
        """envs.step(action) (train.py:151-153): obs, reward, terminated, info
        (device tensors, overwritten by the next call)."""
        a = actions.to(self.device, torch.float32).contiguous()
        _check(load().rt_env_step(self._h, a.data_ptr(), self.obs.data_ptr(), self.reward.data_ptr(),
                                  self.terminated.data_ptr(), self.info.data_ptr(), self._stream()), "rt_env_step")
        return self.obs, self.reward, self.terminated.bool(), self.info

    def close(self):
        if self._h:
            load().rt_env_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
