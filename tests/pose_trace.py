"""Golden rotations under correctly rounded half-angle sin/cos (shared by
tests/test_oracle.py and tests/test_gpu_parity.py)."""
import math

import numpy as np

import oracle as O


def _half_angles(rvs):
    """theta/2 as scipy's from_rotvec computes it (f32 rotvec widened)."""
    r = np.asarray(rvs, np.float64)
    return np.sqrt((r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1]) + r[:, 2] * r[:, 2]) / 2.0


def pose_ulp_trace(z):
    """Per golden rotation: the reference output (libm sin/cos), the oracle
    with correctly rounded half-angle sin/cos (rt_host_sincos, the device's
    rtdd::sincos_cr), and whether libm's sin or cos of theta/2 is off by an ulp."""
    from ppo_radiotherapy_amd import _lib

    L = _lib.load()
    rvs = np.stack([O.map_rotation(a) for a in z["rot_action"]])
    h = _half_angles(rvs)
    s_cr, c_cr = np.zeros_like(h), np.zeros_like(h)
    assert L.rt_host_sincos(len(h), h.ctypes.data, s_cr.ctypes.data, c_cr.ctypes.data) == 0
    libm_off = (np.array([math.sin(v) for v in h]) != s_cr) | (np.array([math.cos(v) for v in h]) != c_cr)
    big = np.linalg.norm(rvs.astype(np.float64), axis=1) > 1e-3  # the small-angle series uses no sin/cos
    libm_off &= big
    cr = np.stack([O.apply_rotation(z["rot_dir_in"][k], rvs[k], half_sincos=(s_cr[k], c_cr[k]))[0]
                   for k in range(len(h))])
    return cr, libm_off
