"""Shared gate of the info doses.lung parity checks (tests only)."""
import numpy as np

# info doses.lung (environment.py:235 = float(np.sum(dose * lungs))).
#
# Dense mode: numpy's exact f32 order (the lung sum plan of csrc/rtenv.hip) --
# bit-exact.
#
# Incremental mode: an f64 running sum of the touched voxels'
# changes, rounded to f32 once.  It is (to ~1e-15) the exact sum S, while the
# reference's f32 np.sum rounds every addition: each term passes through at most
# d additions -- its chain (<= 16), the leaf's tail (<= 7) and 8-accumulator tree
# (3), the buffer's pairwise tree (<= 7 levels) and the sequential fold over the
# ceil(V / 8192) buffers -- and every term is >= 0, so |np.sum - S| <= d * 2^-24 * S
# (+ 1/2 ulp for the final f32 rounding of the f64 sum).  d = 33 + ceil(V / 8192):
# 65 at 64^3 (3.9e-6 relative), 58 at the reference grid.  Measured: up to 6 ulp
# (2.8e-6 at 7.89, tests/test_gpu_headline.py, round 6).
def lung_inc_bound(ref, V=64 ** 3):
    d = 33 + -(-int(V) // 8192)
    return d * 2.0 ** -24 * abs(float(ref)) + 0.5 * float(np.spacing(np.float32(ref)))


def check_dose_lung(got, ref, step_mode, where=None, V=64 ** 3):
    if step_mode == "dense":
        assert np.float32(got) == np.float32(ref), (where, "doses.lung", got, ref)
    else:
        assert abs(float(got) - float(ref)) <= lung_inc_bound(ref, V), (where, "doses.lung", got, ref)
