"""The reference-side binding INTEGRATION.md §2 documents
(INTEGRATION_binding.py, a self-contained ctypes stub over include/rtenv.h)
driven end to end: create, reset with pinned tumours, rt_env_step calls --
against the C oracle (environment.py:77-243 restated), at the reference grid
with the reference tumour library.  The seam is train.py:93-95 (env
construction) and train.py:123,151-158 (reset / step)."""
import os
import sys

import numpy as np
import pytest

import oracle as O
from ppo_radiotherapy_amd import assets

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def test_reference_binding_steps_match_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import INTEGRATION_binding as B

    lib = assets.reference_library()
    vols = [lib.tumour_dense(k) for k in range(lib.n_tumours)]
    tumours = B.tumour_voxels_from_volumes(vols)
    N, T = 8, 24
    env = B.GpuVecEnv(N, lib.lungs, tumours, seed=3)
    rng = np.random.default_rng(7)
    ids = rng.integers(0, lib.n_tumours, N).astype(np.int32)
    obs0 = env.reset(ids).cpu().numpy().copy()
    acts = rng.uniform(-1.1, 1.1, (T, N, 6)).astype(np.float32)
    got = []
    for t in range(T):
        o, r, d, info = env.step(torch.from_numpy(acts[t]))
        got.append((o.cpu().numpy().copy(), r.cpu().numpy().copy(), d.cpu().numpy().copy(),
                    info.cpu().numpy().copy()))
    lungs = lib.lungs.astype(np.float32)
    for e in range(N):
        oe = O.OracleEnv(lungs, lib.tumour_dense(int(ids[e])))
        np.testing.assert_array_equal(obs0[e], oe.reset().astype(np.float32))
        for t in range(T):
            o, info, done = oe.step(acts[t, e])
            np.testing.assert_array_equal(got[t][0][e], o.astype(np.float32), err_msg=f"env {e} step {t}")
            assert abs(got[t][1][e] - info[0]) <= 1e-5
            assert bool(got[t][2][e]) == bool(done)
            np.testing.assert_allclose(got[t][3][e][:4], info[:4], rtol=0, atol=1e-5)
            # doses.tumour / doses.lung: numpy's f32 sums, bit-exact (dense mode)
            assert got[t][3][e][4] == np.float32(info[4]) and got[t][3][e][5] == np.float32(info[5])
            if done:
                break
    env.close()


def test_reference_binding_rejects_stale_struct():
    """A binding whose rt_env_config lacks a member (the round-2 INTEGRATION.md
    snippet had no step_mode) states its own, smaller size: both config calls
    return RT_EINVAL and leave the caller's memory alone."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import ctypes

    import INTEGRATION_binding as B

    L = B.load()

    class Stale(ctypes.Structure):
        _fields_ = B.RtEnvConfig._fields_[:-1]

    buf = (ctypes.c_uint8 * (ctypes.sizeof(B.RtEnvConfig) + 16))()
    ctypes.memset(buf, 0xAB, len(buf))
    cfg = Stale.from_buffer(buf)
    cfg.struct_size = ctypes.sizeof(Stale)
    assert L.rt_env_config_default(ctypes.cast(ctypes.byref(cfg), ctypes.POINTER(B.RtEnvConfig))) == -1
    assert b"struct_size" in L.rt_last_error()
    assert all(b == 0xAB for b in bytes(buf)[4:])
    h = ctypes.c_void_p()
    assert L.rt_env_create(ctypes.cast(ctypes.byref(cfg), ctypes.POINTER(B.RtEnvConfig)), 0, ctypes.byref(h)) == -1
    assert h.value is None
