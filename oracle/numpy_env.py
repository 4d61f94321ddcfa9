"""Op-for-op NumPy restatement of the reference environment step.

TEST INFRASTRUCTURE ONLY (the CPU baseline timed by bench.py and a second
checker for tests/).  It performs the same dense full-volume numpy passes as
the reference -- a Python-loop beam raster (draw_line.py:4-102), scipy's
Rotation (transforms.py:7-59), `np.clip` of the dose, and the reward
reductions with `np.where` scans (environment.py:145-191) -- so its cost per
step tracks the reference's (calibrated in the build container: see
DESIGN.md, "CPU baseline").
"""
from __future__ import annotations

import numpy as np
from scipy.spatial.transform import Rotation

EPS = 1e-6
MIN_ANGLE = np.pi / 4


def _raster(base, pos, direction):
    """Dense f32 beam volume shaped like `base` (draw_line.py:4-102, NEP 50 f32
    arithmetic; the output is allocated like the reference's, zeros_like)."""
    shape = base.shape
    out = np.zeros_like(base, dtype=np.float32)
    p = np.array(pos, dtype=np.float32)
    d = np.array(direction, dtype=np.float32)
    n = np.linalg.norm(d)
    if n < EPS:
        raise ValueError("Direction vector magnitude is too small.")
    d /= n
    lo, hi = [], []
    for ax in range(3):
        if abs(d[ax]) > EPS:
            a = (-p[ax]) / d[ax]
            b = (shape[ax] - 1 - p[ax]) / d[ax]
            lo.append(min(a, b))
            hi.append(max(a, b))
        elif p[ax] < 0 or p[ax] > shape[ax] - 1:
            return out
        else:
            lo.append(-np.inf)
            hi.append(np.inf)
    t0, t1 = max(lo), min(hi)
    if t0 > t1:
        return out
    dom = int(np.argmax(np.abs(d)))
    rest = [ax for ax in range(3) if ax != dom]
    sgn = 1 if d[dom] > 0 else -1
    x = int(np.floor(p[dom] + t0 * d[dom]))
    x_end = int(np.floor(p[dom] + t1 * d[dom]))
    u = p[rest[0]] + t0 * d[rest[0]]
    v = p[rest[1]] + t0 * d[rest[1]]
    du = d[rest[0]] / (d[dom] + EPS)
    dv = d[rest[1]] / (d[dom] + EPS)
    while (x - x_end) * sgn <= 0:
        uf, vf = int(np.floor(u)), int(np.floor(v))
        fu, fv = u - uf, v - vf
        base = [0, 0, 0]
        base[dom], base[rest[0]], base[rest[1]] = x, uf, vf
        for oy, wy in ((0, 1 - fu), (1, fu)):
            for oz, wz in ((0, 1 - fv), (1, fv)):
                i, j, k = base[0], base[1] + oy, base[2] + oz
                if 0 <= i < shape[0] and 0 <= j < shape[1] and 0 <= k < shape[2]:
                    out[i, j, k] += wy * wz
        u += du * sgn
        v += dv * sgn
        x += sgn
    return out


def _rotate(direction, rotvec):
    """transforms.py:7-59."""
    d = direction / np.linalg.norm(direction)
    r = Rotation.from_rotvec(rotvec).apply(d)
    r /= np.linalg.norm(r)
    zc = np.clip(r[0], -1.0, 1.0)
    s = np.sign(zc)
    ang = np.arccos(zc)
    if s < 0:
        ang = np.pi - ang
    if abs(ang) < MIN_ANGLE:
        tz = s * np.cos(MIN_ANGLE)
        txy = np.sqrt(1 - tz ** 2)
        xy = r[1:]
        if np.linalg.norm(xy) < 1e-8:
            xy = np.array([1.0, 0.0])
        else:
            xy /= np.linalg.norm(xy)
        r = np.array([tz, xy[0] * txy, xy[1] * txy])
    r /= np.linalg.norm(r)
    return r, max(0, MIN_ANGLE - ang)


class NumpyEnv:
    """Visionless RadiotherapyEnv dynamics on dense numpy volumes.

    Organised like the reference (environment.py:77-191): one method per
    reward with the same full-volume temporaries and the same lifetimes (a
    temporary lives until its method returns), the dose replaced by a new
    clipped array every step -- so the allocator sees the reference's
    sequence of 806 KB allocations and frees, which decides how many of them
    land on freshly faulted pages (tools/calibrate_cpu.py)."""

    def __init__(self, lungs: np.ndarray, tumour: np.ndarray):
        self.shape = tuple(lungs.shape)
        self.S = np.array(self.shape)
        self.lungs = lungs.astype(np.float32)
        self.set_tumour(tumour)

    def set_tumour(self, tumour):
        """environment.py:86-97: zeros_like + the loaded volume, clipped."""
        vol = np.zeros_like(self.lungs, dtype=np.float32)
        vol += tumour.astype(np.float32)
        self.tumours = np.clip(vol, 0.0, 1.0)

    def reset(self, tumour=None):
        if tumour is not None:
            self.set_tumour(tumour)
        self.pos = self.S / 2
        self.dir = np.array([0.0, 1.0, 0.0])
        self.dose = np.zeros_like(self.lungs, dtype=np.float32)
        self.t = 0
        return self._obs()

    def _tumour_coords(self):
        return np.stack(np.where(self.tumours == 1.0), axis=-1)

    def _obs(self):
        centre = np.mean(self._tumour_coords(), axis=0)
        return np.concatenate([self.pos / self.S * 2 - 1, self.dir, centre / self.S * 2 - 1])

    def _add_beam(self):
        """environment.py:107-110."""
        self.dose += _raster(self.lungs, self.pos, self.dir) * 0.1
        self.dose = np.clip(self.dose, 0.0, 1.0)

    def _tumour_reward(self):
        """environment.py:164-171."""
        on_tumour = self.dose * self.tumours
        got, size = np.sum(on_tumour), np.sum(self.tumours)
        return got / size * 10.0

    def _lung_reward(self):
        """environment.py:173-182."""
        healthy = self.lungs * (1 - self.tumours)
        on_lung = self.dose * healthy
        over = on_lung > 0.2
        n_over, n_lung = np.sum(over), np.sum(healthy)
        return n_over / n_lung * -1.0

    def _distance_reward(self):
        """environment.py:150-162."""
        coords = self._tumour_coords()
        diff = coords - np.array(self.pos)
        dist = np.linalg.norm(diff, axis=1)
        near = diff[np.argmin(dist)]
        return np.linalg.norm(near) / np.linalg.norm(self.S) * -1.0

    def _irradiated(self):
        """environment.py:184-191."""
        on_tumour = self.dose * self.tumours
        got, size = np.sum(on_tumour), np.sum(self.tumours)
        return got / size >= 0.9

    def step(self, action):
        """environment.py:193-243 (info as a flat array: RT_INFO_* order up to 16)."""
        self.t += 1
        tr = np.clip(action[:3], -1.0, 1.0) * self.S * 0.2
        rv = np.clip(action[3:6], -1.0, 1.0) * np.pi * 0.5
        raw = self.pos + tr
        self.pos = np.clip(raw, 0, self.S)
        os_t = np.abs(raw - self.pos)
        self.dir, os_r = _rotate(self.dir, rv)
        self._add_beam()
        r_tum = self._tumour_reward()
        r_lung = self._lung_reward()
        r_dist = self._distance_reward()
        reward = r_tum + r_lung + r_dist
        done = bool(self._irradiated() or self.t >= 100)
        d_tum = float(np.sum(self.dose * self.tumours))
        d_lung = float(np.sum(self.dose * self.lungs))
        info = np.array([reward, r_tum, r_lung, r_dist, d_tum, d_lung, *os_t, os_r, *self.pos, *self.dir])
        return self._obs(), info, done
