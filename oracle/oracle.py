"""ctypes wrapper around oracle/_build/liboracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product package never imports this module.

Each function cites the reference symbol it restates (paths relative to the
reference repo rmaguado/ppo-radiotherapy):

* beam_list / beam_dense     -> draw_line.py:4-102   beam_voxels
* apply_rotation             -> transforms.py:7-59
* apply_translation          -> transforms.py:62-69
* map_translation/rotation   -> environment.py:112-143
* np_sum_f32                 -> numpy np.sum over an f32 volume
                                (environment.py:166-178 reductions)
* OracleEnv                  -> environment.py:15-273  RadiotherapyEnv (visionless)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

INFO_W = 16
MIN_ANGLE_Z = np.pi / 4


def build(force: bool = False) -> str:
    """Compile the C restatement with the committed Makefile."""
    src = os.path.join(_HERE, "rt_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        c_int_p = P(ctypes.c_int)
        d_p = P(ctypes.c_double)
        f_p = P(ctypes.c_float)
        L.or_beam_list.argtypes = [c_int_p, d_p, d_p, P(ctypes.c_int32), f_p, ctypes.c_int]
        L.or_beam_list.restype = ctypes.c_int
        L.or_beam_dense.argtypes = [c_int_p, d_p, d_p, f_p]
        L.or_beam_dense.restype = ctypes.c_int
        L.or_np_sum_f32.argtypes = [f_p, ctypes.c_int64]
        L.or_np_sum_f32.restype = ctypes.c_float
        L.or_apply_rotation.argtypes = [d_p, f_p, ctypes.c_double, d_p, d_p]
        L.or_apply_rotation_sc.argtypes = [d_p, f_p, ctypes.c_double, d_p, d_p, d_p]
        L.or_apply_translation.argtypes = [d_p, d_p, P(ctypes.c_int64), d_p, d_p]
        L.or_map_translation.argtypes = [f_p, P(ctypes.c_int64), d_p]
        L.or_map_rotation.argtypes = [f_p, f_p]
        L.or_env_new.argtypes = [c_int_p, f_p, f_p]
        L.or_env_new.restype = ctypes.c_void_p
        L.or_env_free.argtypes = [ctypes.c_void_p]
        L.or_env_set_tumour.argtypes = [ctypes.c_void_p, f_p]
        L.or_env_reset.argtypes = [ctypes.c_void_p, d_p]
        L.or_env_step.argtypes = [ctypes.c_void_p, f_p, d_p, d_p]
        L.or_env_step.restype = ctypes.c_int
        L.or_env_dose.argtypes = [ctypes.c_void_p]
        L.or_env_dose.restype = f_p
        L.or_env_get_pose.argtypes = [ctypes.c_void_p, d_p, d_p, c_int_p]
        _lib = L
    return _lib


def _ptr(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _shape(shape) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(shape, dtype=np.int32))


def beam_list(shape, pos, direction):
    """Raw splats (flat C-order index int32, weight f32) in reference order.

    Raises ValueError like draw_line.py:23-24 for a near-zero direction."""
    g = _shape(shape)
    cap = 8 * (int(g.sum()) + 4)
    idx = np.zeros(cap, np.int32)
    w = np.zeros(cap, np.float32)
    p = np.ascontiguousarray(pos, dtype=np.float64)
    d = np.ascontiguousarray(direction, dtype=np.float64)
    n = lib().or_beam_list(_ptr(g, ctypes.c_int), _ptr(p, ctypes.c_double), _ptr(d, ctypes.c_double),
                           _ptr(idx, ctypes.c_int32), _ptr(w, ctypes.c_float), cap)
    if n < 0:
        raise ValueError("Direction vector magnitude is too small.")
    return idx[:n].copy(), w[:n].copy()


def beam_dense(shape, pos, direction) -> np.ndarray:
    g = _shape(shape)
    out = np.zeros(int(np.prod(g)), np.float32)
    p = np.ascontiguousarray(pos, dtype=np.float64)
    d = np.ascontiguousarray(direction, dtype=np.float64)
    rc = lib().or_beam_dense(_ptr(g, ctypes.c_int), _ptr(p, ctypes.c_double), _ptr(d, ctypes.c_double),
                             _ptr(out, ctypes.c_float))
    if rc < 0:
        raise ValueError("Direction vector magnitude is too small.")
    return out.reshape(tuple(int(x) for x in g))


def beam_sparse(shape, pos, direction):
    """Sorted unique nonzero voxels of the dense beam: (flat idx int32, f32)."""
    dense = beam_dense(shape, pos, direction).ravel()
    nz = np.flatnonzero(dense).astype(np.int32)
    return nz, dense[nz]


def np_sum_f32(a: np.ndarray) -> np.float32:
    a = np.ascontiguousarray(a, dtype=np.float32).ravel()
    return np.float32(lib().or_np_sum_f32(_ptr(a, ctypes.c_float), a.size))


def apply_rotation(direction, rotvec, min_angle=MIN_ANGLE_Z, half_sincos=None):
    """transforms.py:7-59.  half_sincos: None = libm sin/cos of theta/2 (as
    scipy's from_rotvec); else (sin, cos) of theta/2 to use instead."""
    d = np.ascontiguousarray(direction, dtype=np.float64)
    r = np.ascontiguousarray(rotvec, dtype=np.float32)
    out = np.zeros(3, np.float64)
    os_ = np.zeros(1, np.float64)
    sc = None if half_sincos is None else np.ascontiguousarray(half_sincos, dtype=np.float64)
    lib().or_apply_rotation_sc(_ptr(d, ctypes.c_double), _ptr(r, ctypes.c_float), float(min_angle),
                               None if sc is None else _ptr(sc, ctypes.c_double),
                               _ptr(out, ctypes.c_double), _ptr(os_, ctypes.c_double))
    return out, float(os_[0])


def apply_translation(pos, tr, bounds):
    p = np.ascontiguousarray(pos, dtype=np.float64)
    t = np.ascontiguousarray(tr, dtype=np.float64)
    b = np.ascontiguousarray(bounds, dtype=np.int64)
    out = np.zeros(3, np.float64)
    os_ = np.zeros(3, np.float64)
    lib().or_apply_translation(_ptr(p, ctypes.c_double), _ptr(t, ctypes.c_double),
                               _ptr(b, ctypes.c_int64), _ptr(out, ctypes.c_double), _ptr(os_, ctypes.c_double))
    return out, os_


def map_translation(a, shape):
    a = np.ascontiguousarray(a, dtype=np.float32)
    S = np.ascontiguousarray(shape, dtype=np.int64)
    out = np.zeros(3, np.float64)
    lib().or_map_translation(_ptr(a, ctypes.c_float), _ptr(S, ctypes.c_int64), _ptr(out, ctypes.c_double))
    return out


def map_rotation(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    out = np.zeros(3, np.float32)
    lib().or_map_rotation(_ptr(a, ctypes.c_float), _ptr(out, ctypes.c_float))
    return out


class OracleEnv:
    """Single visionless env with dense volumes (environment.py:15-273).

    The tumour is supplied explicitly as a dense f32 {0,1} volume; the
    reference draws it with np.random.choice (environment.py:90)."""

    def __init__(self, lungs: np.ndarray, tumour: np.ndarray):
        self.shape = tuple(int(x) for x in lungs.shape)
        self._g = _shape(self.shape)
        self._lungs = np.ascontiguousarray(lungs, dtype=np.float32).ravel().copy()
        self._tumour = np.ascontiguousarray(tumour, dtype=np.float32).ravel().copy()
        self._h = lib().or_env_new(_ptr(self._g, ctypes.c_int), _ptr(self._lungs, ctypes.c_float),
                                   _ptr(self._tumour, ctypes.c_float))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            lib().or_env_free(h)
            self._h = None

    def set_tumour(self, tumour: np.ndarray):
        self._tumour = np.ascontiguousarray(tumour, dtype=np.float32).ravel().copy()
        lib().or_env_set_tumour(self._h, _ptr(self._tumour, ctypes.c_float))

    def reset(self, tumour: np.ndarray | None = None):
        if tumour is not None:
            self.set_tumour(tumour)
        obs = np.zeros(9, np.float64)
        lib().or_env_reset(self._h, _ptr(obs, ctypes.c_double))
        return obs

    def step(self, action):
        a = np.ascontiguousarray(action, dtype=np.float32)
        obs = np.zeros(9, np.float64)
        info = np.zeros(INFO_W, np.float64)
        done = lib().or_env_step(self._h, _ptr(a, ctypes.c_float), _ptr(obs, ctypes.c_double),
                                 _ptr(info, ctypes.c_double))
        return obs, info, bool(done)

    @property
    def dose(self) -> np.ndarray:
        V = int(np.prod(self.shape))
        p = lib().or_env_dose(self._h)
        return np.ctypeslib.as_array(p, shape=(V,)).copy().reshape(self.shape)

    def pose(self):
        pos = np.zeros(3, np.float64)
        d = np.zeros(3, np.float64)
        t = ctypes.c_int(0)
        lib().or_env_get_pose(self._h, _ptr(pos, ctypes.c_double), _ptr(d, ctypes.c_double), ctypes.byref(t))
        return pos, d, t.value
