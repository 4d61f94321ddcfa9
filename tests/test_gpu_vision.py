"""Vision observations (environment.py:245-257) from the HIP path vs the
reference's get_volumes() (golden) and the oracle's beam rasteriser."""
import numpy as np
import pytest

import oracle as O
from ppo_radiotherapy_amd import assets

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _sparse(ch):
    f = ch.ravel()
    nz = np.flatnonzero(f)
    return nz, f[nz]


def test_vision_obs_matches_reference_get_volumes(golden):
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    z = golden("vision_obs.npz")
    lib = assets.reference_library()
    env = RadiotherapyVecEnv(2, visionless=False, library=lib)
    tid = int(z["tumour_id"])
    obs, _ = env.reset(options={"tumour_ids": np.array([tid, tid], np.int32)})
    assert tuple(obs.shape) == (2, 4, 67, 43, 70)
    lungs = lib.lungs.astype(np.float32)
    tum = lib.tumour_dense(tid)
    for k in range(4):
        if k > 0:
            a = torch.tensor(np.stack([z["actions"][k - 1]] * 2), device=env.device)
            obs, *_ = env.step(a)
        o = obs[0].cpu().numpy()
        np.testing.assert_array_equal(o[0], lungs)
        np.testing.assert_array_equal(o[1], tum)
        lo, hi = z["dose_off"][k], z["dose_off"][k + 1]
        i, v = _sparse(o[2])
        np.testing.assert_array_equal(i, z["dose_idx"][lo:hi])
        np.testing.assert_array_equal(v, z["dose_val"][lo:hi])
        lo, hi = z["view_off"][k], z["view_off"][k + 1]
        i, v = _sparse(o[3])
        np.testing.assert_array_equal(i, z["view_idx"][lo:hi])
        np.testing.assert_array_equal(v.view(np.uint32), z["view_val"][lo:hi].view(np.uint32))
        np.testing.assert_array_equal(obs[1].cpu().numpy(), o)
        sums = o.astype(np.float64).reshape(4, -1).sum(1)
        np.testing.assert_allclose(sums, z["channel_sums"][k], rtol=1e-9)
    env.close()


def test_vision_view_64_vs_oracle():
    """Beam-view channel at 64^3 on random poses: clip(beam(p,d) + beam(p,[1,0,0]))."""
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    lib = assets.synthetic_library((64, 64, 64), 32, 0)
    N = 16
    env = RadiotherapyVecEnv(N, visionless=False, library=lib)
    env.reset(options={"tumour_ids": np.arange(N, dtype=np.int32)})
    rng = np.random.default_rng(0)
    pose = np.zeros((N, 6))
    pose[:, :3] = rng.uniform(0, 64, (N, 3))
    d = rng.normal(size=(N, 3))
    pose[:, 3:] = d / np.linalg.norm(d, axis=1, keepdims=True)
    pose[0, :3] = [64.0, 63.0, 0.0]  # on the clip bounds
    env.set_pose(torch.tensor(pose))
    obs, _ = env.reset(options={"mask": np.zeros(N, bool)})  # NOOP: re-emit the observation
    o = obs.cpu().numpy()
    for e in range(N):
        b1 = O.beam_dense((64, 64, 64), pose[e, :3], pose[e, 3:])
        b2 = O.beam_dense((64, 64, 64), pose[e, :3], np.array([1.0, 0.0, 0.0]))
        view = np.clip(b1 + b2, 0.0, 1.0)
        np.testing.assert_array_equal(o[e, 3].view(np.uint32), view.view(np.uint32), err_msg=f"env {e}")
        np.testing.assert_array_equal(o[e, 0], lib.lungs.astype(np.float32))
    env.close()


def test_vision_large_batch_rewards_match_visionless():
    """Vision mode computes the same dynamics/rewards as the visionless env."""
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    lib = assets.synthetic_library((64, 64, 64), 1000, 0)
    N = 128
    ev = RadiotherapyVecEnv(N, visionless=False, library=lib, seed=9)
    el = RadiotherapyVecEnv(N, visionless=True, library=lib, seed=9)
    ids = (np.arange(N) * 7 % 1000).astype(np.int32)
    ev.reset(options={"tumour_ids": ids})
    el.reset(options={"tumour_ids": ids})
    rng = np.random.default_rng(1)
    for t in range(20):
        a = torch.tensor(rng.uniform(-1, 1, (N, 6)).astype(np.float32), device=ev.device)
        ov, rv, tv, _, _ = ev.step(a)
        ol, rl, tl, _, _ = el.step(a)
        assert torch.equal(rv, rl) and torch.equal(tv, tl)
    torch.testing.assert_close(ev.dose(), el.dose(), rtol=0, atol=0)
    torch.testing.assert_close(ov[:, 2], ev.dose(), rtol=0, atol=0)
    ev.close()
    el.close()
