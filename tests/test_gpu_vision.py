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


def test_render_reproduces_observations():
    """Compact vision storage: observations re-rendered from
    (dose, pose, tumour) snapshots equal the emitted ones bit for bit,
    including across the t = 100 truncation autoreset."""
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    N = 4
    env = RadiotherapyVecEnv(N, visionless=False, seed=5)
    obs, _ = env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    keep = {0, 1, 2, 37, 99, 100, 101, 104}
    V = int(np.prod(env.grid))
    snaps, seen = [], []
    for t in range(105):
        if t in keep:
            d = torch.empty((N, V), device="cuda")
            p = torch.empty((N, 6), dtype=torch.float64, device="cuda")
            k = torch.empty(N, dtype=torch.int32, device="cuda")
            env.snapshot(d, p, k)
            snaps.append((d, p, k))
            seen.append(obs.clone())
        a = torch.rand((N, 6), device="cuda", generator=g) * 2 - 1
        obs, _, _, _, _ = env.step(a)
    dd = torch.cat([s[0] for s in snaps])
    pp = torch.cat([s[1] for s in snaps])
    kk = torch.cat([s[2] for s in snaps])
    r = env.render(dd, pp, kk)
    torch.cuda.synchronize()
    assert torch.equal(r, torch.cat(seen))
    env.close()


def test_compact_trainer_sees_stored_observations():
    """A trainer with compact storage renders exactly the observations a
    trainer with full [T, N, 4, V] storage keeps, and computes the same loss."""
    from types import SimpleNamespace

    from ppo_radiotherapy_amd.networks import PPO_3DCNN
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    out = {}
    for compact in (False, True):
        env = RadiotherapyVecEnv(6, visionless=False, seed=2)
        torch.manual_seed(0)
        agent = PPO_3DCNN((4, *env.grid), (6,), 64).cuda()
        cfg = SimpleNamespace(num_steps=5, num_minibatches=2, update_epochs=1, learning_rate=3e-4, anneal_lr=False,
                              gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True,
                              ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, compact_vision_rollout=compact,
                              micro_batch=8)
        tr = PPOTrainer(cfg, env, agent, "cuda", generator=torch.Generator(device="cuda").manual_seed(1))
        assert tr.compact_obs == compact
        tr.reset()
        tr.rollout()
        tr.compute_gae()
        tr._bind_batch()
        rows = torch.arange(tr.batch_size, device="cuda")
        out[compact] = (tr._obs_rows(rows).clone(), tr._loss_backward(rows).cpu())
        env.close()
    assert torch.equal(out[True][0], out[False][0])
    torch.testing.assert_close(out[True][1], out[False][1], rtol=0, atol=0)


def test_render_from_store_rows_matches_copied_doses():
    """The trainer's render path (rt_env_set_render_source: the reset reads
    each state's dose straight from its row of the dose store) re-emits the
    same observations bit for bit as rendering from copied doses.  32^3 grid:
    rows of exactly the padded volume, so the store path is taken."""
    from ppo_radiotherapy_amd import assets
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    lib = assets.synthetic_library((32, 32, 32), 50, 0)
    N = 8
    env = RadiotherapyVecEnv(N, visionless=False, library=lib, seed=3)
    env.reset()
    g = torch.Generator(device="cuda").manual_seed(0)
    V = int(np.prod(env.grid))
    ds, ps, ks = [], [], []
    for t in range(6):
        d = torch.empty((N, V), device="cuda")
        p = torch.empty((N, 6), dtype=torch.float64, device="cuda")
        k = torch.empty(N, dtype=torch.int32, device="cuda")
        env.snapshot(d, p, k)
        ds.append(d)
        ps.append(p)
        ks.append(k)
        env.step(torch.rand((N, 6), device="cuda", generator=g) * 2 - 1)
    store, pose, tum = torch.cat(ds), torch.cat(ps), torch.cat(ks)
    rows = torch.randperm(store.shape[0], device="cuda", generator=g)[:13]
    via_store = env.render(store, pose[rows], tum[rows], rows=rows).clone()
    assert getattr(env, "_render_rows", None) is not None  # the store path ran
    copied = env.render(store[rows], pose[rows], tum[rows])
    torch.cuda.synchronize()
    assert torch.equal(via_store, copied)
    env.close()
