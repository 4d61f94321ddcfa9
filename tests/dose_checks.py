"""Shared gate of the info doses.lung parity checks (tests only)."""
import numpy as np

# info doses.lung (environment.py:235 = float(np.sum(dose * lungs))).  Dense
# mode: numpy's exact f32 order (the lung sum plan) -- bit-exact.  Incremental
# mode: an f64 running sum rounded once, so it may differ from
# numpy's f32 pairwise sum by that sum's own rounding: gated at 4 ulp of the
# f32 value (<= 1.2e-4 absolute at the ~470 maximum of these fixtures; 1 ulp
# measured on the reference trajectories' final doses).
LUNG_INC_ULPS = 4


def check_dose_lung(got, ref, step_mode, where=None):
    if step_mode == "dense":
        assert np.float32(got) == np.float32(ref), (where, "doses.lung", got, ref)
    else:
        assert abs(float(got) - float(ref)) <= LUNG_INC_ULPS * float(np.spacing(np.float32(ref))), \
            (where, "doses.lung", got, ref)
