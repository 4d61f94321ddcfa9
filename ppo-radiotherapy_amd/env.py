"""Single-env facade with the reference's `RadiotherapyEnv` surface
(environment.py:15-303): `reset(seed, options) -> (obs, {})`,
`step(action) -> (obs, reward, terminated, False, info)` with numpy in/out.

It is a RadiotherapyVecEnv with N = 1 plus host copies, for the callers that
use the env one step at a time (ppo_eval.py, ppo_visualize.py, human_play).
Every step runs the HIP kernels; values are read back from the device (one
sync per step, which the vectorised trainer never pays).

Tumour selection follows the reference: `np.random.choice(TUMOUR_DIRS)` on
the global numpy RNG (environment.py:90), with TUMOUR_DIRS in the build
container's os.listdir order, so a given `np.random.seed` picks the same
tumours as the reference.
"""
from __future__ import annotations

import numpy as np
import torch

from . import assets, spaces
from .vec_env import RadiotherapyVecEnv


class RadiotherapyEnv:
    ACTION_SIZE = 6
    MAX_TIME_STEPS = 100
    MIN_ANGLE_Z = np.pi / 4
    BEAM_DOSE = 0.1
    LUNG_DOSE_THRESHOLD = 0.2
    TUMOUR_DOSE_THRESHOLD = 0.9
    LUNG_DOSE_REWARD = -1.0
    TUMOUR_DOSE_REWARD = 10.0
    DISTANCE_TO_TUMOUR_REWARD = -1.0
    MOVEMENT_SPEED = 0.2
    ROTATION_SPEED = 0.5

    metadata = {"render_modes": ["human"], "render_fps": 30}

    def __init__(self, visionless: bool = False, grid=None, device=None, library=None):
        self.library = library if library is not None else assets.library_for(grid or (67, 43, 70))
        self.TUMOUR_DIRS = list(self.library.names)
        self.LUNGS_ARRAY = self.library.lungs.astype(np.float32)
        self.LUNG_SHAPE = np.array(self.library.shape)
        self.visionless = visionless
        self._vec = RadiotherapyVecEnv(1, visionless=visionless, library=self.library, device=device)
        self.lungs = np.copy(self.LUNGS_ARRAY)
        self.tumours = None
        self.tumours_meta = []
        self.beams = []
        self.t = 0
        self.done = False
        self._tumour_id = -1
        self._last_info = None
        self.reset()
        self.observation_shape = (9,) if visionless else (4, *self.LUNG_SHAPE)
        self.observation_space = spaces.Box(0.0, 1.0, self.observation_shape, np.float32)
        self.action_space = spaces.Box(-1.0, 1.0, (self.ACTION_SIZE,), np.float32)
        self.max_episode_steps = self.MAX_TIME_STEPS

    # ------------------------------------------------------------------ gym API
    def reset(self, seed=None, options=None):
        """environment.py:77-84 (the reference ignores `seed`; so does this)."""
        options = options or {}
        if "tumour_id" in options:
            tid = int(options["tumour_id"])
        else:
            tid = int(np.random.choice(len(self.TUMOUR_DIRS)))
        self._tumour_id = tid
        name = self.TUMOUR_DIRS[tid]
        self.tumours = self.library.tumour_dense(tid)
        attrs = name.split(".npy")[0].split("_")
        self.tumours_meta = [(np.array(attrs[:3], dtype=np.float32), float(attrs[3]))]
        self._vec.reset(options={"tumour_ids": np.array([tid], np.int32)})
        self.beams = []
        self.t = 0
        self.done = False
        self._last_info = None
        self._sync_pose()
        return self.observation(), {}

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, self.ACTION_SIZE),
                            device=self._vec.device)
        obs, rew, term, _, _ = self._vec.step(a)
        info_row = self._vec.info[0].cpu().numpy()
        self._last_info = info_row
        self.t += 1
        self._sync_pose()
        self.beams.append((self.beam_position.copy(), self.beam_direction.copy()))
        self.done = bool(term[0].item())
        info = {
            "reward_components": {
                "total": float(info_row[0]), "tumour": float(info_row[1]), "lung": float(info_row[2]),
                "distance_to_tumour": float(info_row[3]),
            },
            "beam_position": {"translation": list(self.beam_position), "rotation": list(self.beam_direction)},
            "doses": {"tumour": float(info_row[4]), "lung": float(info_row[5])},
            "overshoot": {"translation": list(info_row[6:9].astype(np.float64)), "rotation": float(info_row[9])},
        }
        return self.observation(), float(info_row[0]), self.done, False, info

    # ------------------------------------------------------------------ state
    def _sync_pose(self):
        pose, t, _ = self._vec.get_state()
        p = pose[0].cpu().numpy()
        self.beam_position = p[:3].copy()
        self.beam_direction = p[3:].copy()

    @property
    def dose(self) -> np.ndarray:
        return self._vec.dose()[0].cpu().numpy()

    def tumour_position(self):
        """environment.py:145-148."""
        return self.library.centroid(self._tumour_id)

    def get_vector_observation(self):
        """environment.py:259-268, f64 as the reference returns it."""
        S = self.LUNG_SHAPE
        return np.concatenate([self.beam_position / S * 2 - 1, self.beam_direction,
                               self.tumour_position() / S * 2 - 1])

    def observation(self):
        if self.visionless:
            return self.get_vector_observation()
        return self._vec.obs[0].cpu().numpy()

    def _info_value(self, k):
        if self._last_info is None:
            raise RuntimeError("no step taken since reset")
        return float(self._last_info[k])

    def tumour_dose_reward(self):
        return self._info_value(1)

    def lungs_dose_reward(self):
        return self._info_value(2)

    def distance_to_tumour_reward(self):
        return self._info_value(3)

    def is_fully_irradiated(self):
        return self.tumour_dose_reward() / self.TUMOUR_DOSE_REWARD >= np.float32(self.TUMOUR_DOSE_THRESHOLD)

    def export_trajectory(self, filename):
        """environment.py:69-75 (same npz keys)."""
        np.savez_compressed(filename, tumours=self.tumours, dose=self.dose,
                            beams=np.array(self.beams, dtype=np.float64))

    # ------------------------------------------------------------------ out of scope
    def render(self):
        raise NotImplementedError("rendering (graphics.py, trimesh) is outside this framework's scope")

    def export_animation(self, output_file=None):
        raise NotImplementedError("animation export (graphics.py, trimesh) is outside this framework's scope")

    def inspect_volumes(self):
        raise NotImplementedError("the matplotlib slice viewer is outside this framework's scope")

    def close(self):
        self._vec.close()
