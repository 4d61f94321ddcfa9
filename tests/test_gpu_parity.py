"""HIP path vs the reference (golden vectors) and the C oracle.

Bars: beam voxel lists bit-exact; transforms f64 bit-exact
(overshoot.rotation within 1e-12: acos differs by an ulp between numpy's SVML,
libm and ocml); env obs/reward/doses within 1e-5 (fp32), done identical,
accumulated dose volumes bit-exact.
"""
import ctypes

import time

import numpy as np
import pytest

import oracle as O
from ppo_radiotherapy_amd import _lib, assets

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


def _vec_env(n, library, seed=0, step_mode="dense"):
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    return RadiotherapyVecEnv(n, visionless=True, library=library, seed=seed, step_mode=step_mode)


MODES = ["dense", "incremental"]


from dose_checks import check_dose_lung, lung_inc_bound  # noqa: E402


# ----------------------------------------------------------------- beams
def test_beam_cases_bit_exact(golden, dev):
    z = golden("beam_cases.npz")
    L = _lib.load()
    off = z["offsets"]
    grids = z["grid"]
    for g in np.unique(grids, axis=0):
        sel = np.flatnonzero((grids == g).all(axis=1))
        m = len(sel)
        cap = 8 * (int(g.sum()) + 4)
        pos = torch.tensor(z["pos"][sel], dtype=torch.float64, device=dev)
        dr = torch.tensor(z["dir"][sel], dtype=torch.float64, device=dev)
        idx = torch.zeros((m, cap), dtype=torch.int32, device=dev)
        w = torch.zeros((m, cap), dtype=torch.float32, device=dev)
        cnt = torch.zeros(m, dtype=torch.int32, device=dev)
        _lib.check(L.rt_debug_beam(_lib.grid_arg(g), m, pos.data_ptr(), dr.data_ptr(), cap, idx.data_ptr(),
                                   w.data_ptr(), cnt.data_ptr(), None), "rt_debug_beam")
        torch.cuda.synchronize()
        idx, w, cnt = idx.cpu().numpy(), w.cpu().numpy(), cnt.cpu().numpy()
        V = int(np.prod(g))
        for r, k in enumerate(sel):
            if z["err"][k]:
                assert cnt[r] == -1
                continue
            # accumulate raw splats exactly like `output[ix,iy,iz] += weight`
            dense = np.zeros(V, np.float32)
            for i in range(cnt[r]):
                dense[idx[r, i]] = np.float32(dense[idx[r, i]] + w[r, i])
            nz = np.flatnonzero(dense)
            assert np.array_equal(nz, z["idx"][off[k]:off[k + 1]]), (g, k)
            assert np.array_equal(dense[nz].view(np.uint32), z["val"][off[k]:off[k + 1]].view(np.uint32)), (g, k)


def test_pose_cases(golden, dev):
    z = golden("transform_cases.npz")
    L = _lib.load()
    m = len(z["rot_action"])
    # rotation cases: pos unchanged (zero translation action), dir/rotvec from the fixture
    pos = np.tile(np.array([33.5, 21.5, 35.0]), (m, 1))
    act = np.zeros((m, 6), np.float32)
    act[:, 3:] = z["rot_action"]
    out = _run_pose(L, dev, (67, 43, 70), pos, z["rot_dir_in"], act)
    # scipy's from_rotvec takes sin/cos of theta/2 from libm; the kernel
    # evaluates them correctly rounded (rtdd::sincos_cr).  Gate: the kernel is
    # bit-exact against the oracle fed the correctly rounded half-angle sin/cos
    # on EVERY rotation, and differs from the reference only on the rotations
    # whose glibc sin or cos is itself 1 ulp off (5 of 3000; traced in
    # tests/test_oracle.py::test_pose_ulp_differences_trace_to_libm_sincos).
    from pose_trace import pose_ulp_trace

    got, want = out[:, 3:6], z["rot_dir_out"]
    cr, libm_off = pose_ulp_trace(z)
    assert np.array_equal(got.view(np.int64), cr.view(np.int64))
    differs = ~np.all(got == want, axis=1)
    assert not np.any(differs & ~libm_off)
    assert np.abs(got - want).max() <= 1e-15
    assert np.max(np.abs(out[:, 9] - z["rot_overshoot"])) <= 1e-12
    # translation cases
    act = np.zeros((m, 6), np.float32)
    act[:, :3] = z["tr_action"]
    dirs = np.tile(np.array([0.0, 1.0, 0.0]), (m, 1))
    out = _run_pose(L, dev, tuple(z["tr_bounds"]), z["tr_pos_in"], dirs, act)
    assert np.array_equal(out[:, 0:3], z["tr_pos_out"])
    assert np.array_equal(out[:, 6:9], z["tr_overshoot"])


def _run_pose(L, dev, grid, pos, dirs, act):
    m = len(pos)
    p = torch.tensor(np.asarray(pos), dtype=torch.float64, device=dev)
    d = torch.tensor(np.asarray(dirs), dtype=torch.float64, device=dev)
    a = torch.tensor(np.asarray(act), dtype=torch.float32, device=dev)
    out = torch.zeros((m, 10), dtype=torch.float64, device=dev)
    _lib.check(L.rt_debug_pose(_lib.grid_arg(grid), m, p.data_ptr(), d.data_ptr(), a.data_ptr(), out.data_ptr(),
                               None), "rt_debug_pose")
    torch.cuda.synchronize()
    return out.cpu().numpy()


# ----------------------------------------------------------------- env trajectories
def _replay(z, lib, tol=1e-5, step_mode="dense"):
    n_eps = len(z["tumour_id"])
    env = _vec_env(n_eps, lib, step_mode=step_mode)
    obs, _ = env.reset(options={"tumour_ids": z["tumour_id"].astype(np.int32)})
    np.testing.assert_array_equal(obs.cpu().numpy(), z["obs0"].astype(np.float32))
    lens = z["ep_len"]
    offs = np.concatenate([[0], np.cumsum(lens)])
    T = int(lens.max())
    acts = torch.tensor(z["actions"], dtype=torch.float32, device=env.device)  # [E, 100, 6]
    worst = 0.0
    for t in range(T):
        obs, rew, term, trunc, infos = env.step(acts[:, t].contiguous())
        o = obs.cpu().numpy()
        r = rew.cpu().numpy()
        rc = {k: infos["reward_components"][k].cpu().numpy() for k in ("tumour", "lung", "distance_to_tumour")}
        dz = {k: infos["doses"][k].cpu().numpy() for k in ("tumour", "lung")}
        term = term.cpu().numpy()
        for e in range(n_eps):
            if t >= lens[e]:
                continue
            k = offs[e] + t
            np.testing.assert_array_equal(o[e], z["step_obs"][k].astype(np.float32), err_msg=f"ep {e} t {t}")
            assert abs(r[e] - z["step_reward"][k]) <= tol
            assert abs(rc["tumour"][e] - z["step_tumour"][k]) <= tol
            assert abs(rc["lung"][e] - z["step_lung"][k]) <= tol
            assert abs(rc["distance_to_tumour"][e] - z["step_dist"][k]) <= tol
            assert dz["tumour"][e] == np.float32(z["step_dose_tumour"][k])
            check_dose_lung(dz["lung"][e], z["step_dose_lung"][k], step_mode, (e, t), lib.V)
            assert bool(term[e]) == bool(z["step_done"][k]), f"ep {e} t {t}"
            worst = max(worst, abs(r[e] - z["step_reward"][k]))
        if t == T - 1 or np.any(lens == t + 1):
            dose = env.dose().cpu().numpy().reshape(n_eps, -1)
            for e in np.flatnonzero(lens == t + 1):
                lo, hi = z["dose_off"][e], z["dose_off"][e + 1]
                nz = np.flatnonzero(dose[e])
                np.testing.assert_array_equal(nz, z["dose_idx"][lo:hi])
                np.testing.assert_array_equal(dose[e][nz].view(np.uint32), z["dose_val"][lo:hi].view(np.uint32))
    env.close()
    return worst


@pytest.mark.parametrize("mode", MODES)
def test_env_trajectories_reference_grid(golden, dev, mode):
    _replay(golden("env_traj_ref.npz"), assets.reference_library(), step_mode=mode)


@pytest.mark.parametrize("mode", MODES)
def test_env_trajectories_64(golden, dev, mode):
    _replay(golden("env_traj_64.npz"), assets.synthetic_library((64, 64, 64), 64, 0), step_mode=mode)


def _custom_library(shape, lungs, tumours):
    vox = [np.sort(np.asarray(t, np.int32)) for t in tumours]
    off = np.concatenate([[0], np.cumsum([len(v) for v in vox])]).astype(np.int64)
    return assets.TumourLibrary(shape=tuple(shape), lungs=lungs.astype(np.uint8), names=[str(i) for i in range(len(vox))],
                                voxels=np.concatenate(vox), offsets=off)


@pytest.mark.parametrize("mode", MODES)
def test_termination_and_autoreset(golden, dev, mode):
    """Episodes ending by irradiation (environment.py:184-191,220) followed by
    gymnasium NEXT_STEP autoreset and RecordEpisodeStatistics."""
    z = golden("env_done_ref.npz")
    ref = assets.reference_library()
    tumours = []
    for e in range(len(z["len"])):
        vv = [int(np.ravel_multi_index(tuple(v), ref.shape)) for v in z["tumour_vox"][e] if v[0] >= 0]
        tumours.append(vv)
    lib = _custom_library(ref.shape, ref.lungs, tumours)
    E = len(tumours)
    env = _vec_env(E, lib, step_mode=mode)
    t_start = time.perf_counter()  # the envs' RecordEpisodeStatistics clocks start inside reset()
    env.reset(options={"tumour_ids": np.arange(E, dtype=np.int32)})
    acts = torch.tensor(z["actions"], dtype=torch.float32, device=env.device)
    ret = np.zeros(E)
    finished = np.zeros(E, bool)
    for t in range(101):
        a = acts[:, min(t, 99)].contiguous()
        obs, rew, term, trunc, infos = env.step(a)
        t_now = time.perf_counter()
        r = rew.cpu().numpy()
        term = term.cpu().numpy()
        stepped = infos["_reward_components"].cpu().numpy()
        epd = infos["_episode"].cpu().numpy()
        for e in range(E):
            L = int(z["len"][e])
            if t < L:
                assert stepped[e]
                assert abs(r[e] - z["reward"][e][t]) <= 1e-5
                assert bool(term[e]) == bool(z["done"][e][t])
                ret[e] += z["reward"][e][t]
                if t == L - 1:
                    assert epd[e]
                    assert abs(infos["episode"]["r"][e].item() - ret[e]) <= 1e-4
                    assert infos["episode"]["l"][e].item() == L
                    # episode["t"] (gymnasium 1.0 RecordEpisodeStatistics): wall
                    # seconds since the env's reset, rounded to 6 decimals
                    ep_t = infos["episode"]["t"][e].item()
                    assert infos["episode"]["_t"][e].item()
                    assert 0.0 < ep_t <= t_now - t_start + 1e-6 and abs(ep_t - round(ep_t, 6)) < 1e-9
                    finished[e] = True
            elif t == L:  # autoreset step: action ignored, reward 0, reset obs
                assert not stepped[e] and r[e] == 0.0 and not term[e] and not epd[e]
                o = obs[e].cpu().numpy()
                np.testing.assert_array_equal(o[:6], np.array([0, 0, 0, 0, 1, 0], np.float32))
    assert finished.all()
    env.close()


def test_large_batch_vs_oracle(dev):
    """4096 envs at 64^3 (BASELINE config 2): a sample of envs replayed on the
    oracle must match bit-exactly in dose and within 1e-5 in reward."""
    lib = assets.synthetic_library((64, 64, 64), 1000, 0)
    N = 4096
    env = _vec_env(N, lib, seed=123)
    rng = np.random.default_rng(0)
    ids = rng.integers(0, lib.n_tumours, N).astype(np.int32)
    env.reset(options={"tumour_ids": ids})
    T = 12
    acts = rng.uniform(-1.1, 1.1, (T, N, 6)).astype(np.float32)
    rewards = []
    for t in range(T):
        _, rew, term, _, _ = env.step(torch.tensor(acts[t], device=env.device))
        rewards.append(rew.cpu().numpy().copy())
    dose = env.dose()
    sample = [0, 1, 777, 2048, 4095]
    lungs = lib.lungs.astype(np.float32)
    for e in sample:
        oe = O.OracleEnv(lungs, lib.tumour_dense(int(ids[e])))
        oe.reset()
        for t in range(T):
            _, info, _ = oe.step(acts[t, e])
            assert abs(rewards[t][e] - info[0]) <= 1e-5
        got = dose[e].cpu().numpy()
        np.testing.assert_array_equal(got.view(np.uint32), oe.dose.view(np.uint32))
    env.close()


# ----------------------------------------------------------------- GAE
@pytest.mark.parametrize("T,N", [(37, 513), (64, 4096), (1, 3), (2048, 16)])
def test_gae_matches_torch_loop(dev, T, N):
    """rt_gae (the reverse scan loading kGaeChunk steps ahead, ragged last
    chunk) vs train.py:163-181's loop."""
    g = torch.Generator(device="cpu").manual_seed(0)
    rew = torch.randn(T, N, generator=g).to(dev)
    val = torch.randn(T, N, generator=g).to(dev)
    dones = (torch.rand(T, N, generator=g) < 0.1).float().to(dev)
    nv = torch.randn(N, generator=g).to(dev)
    nd = (torch.rand(N, generator=g) < 0.1).float().to(dev)
    gamma, lam = 0.99, 0.95
    # train.py:163-181 verbatim semantics
    adv_ref = torch.zeros_like(rew)
    last = 0
    for t in reversed(range(T)):
        if t == T - 1:
            nnt, nvals = 1.0 - nd, nv
        else:
            nnt, nvals = 1.0 - dones[t + 1], val[t + 1]
        delta = rew[t] + gamma * nvals * nnt - val[t]
        adv_ref[t] = last = delta + gamma * lam * nnt * last
    ret_ref = adv_ref + val
    adv = torch.empty_like(rew)
    ret = torch.empty_like(rew)
    L = _lib.load()
    _lib.check(L.rt_gae(T, N, rew.data_ptr(), val.data_ptr(), dones.data_ptr(), nv.data_ptr(), nd.data_ptr(),
                        gamma, lam, adv.data_ptr(), ret.data_ptr(), None), "rt_gae")
    torch.testing.assert_close(adv, adv_ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(ret, ret_ref, rtol=1e-6, atol=1e-6)


def test_incremental_equals_dense_over_resets(dev):
    """4096 envs at 64^3 for 230 steps (>= 2 episodes each, Philox tumour draws):
    the incremental step gives bitwise the same rewards, termination and dose
    as the dense step; doses.lung (the dense mode's is numpy's exact f32 sum)
    within the incremental mode's rounding bound (tests/dose_checks.py)."""
    lib = assets.synthetic_library((64, 64, 64), 1000, 0)
    N = 4096
    d = _vec_env(N, lib, seed=11, step_mode="dense")
    i = _vec_env(N, lib, seed=11, step_mode="incremental")
    d.reset()
    i.reset()
    g = torch.Generator(device=d.device).manual_seed(0)
    for t in range(230):
        a = torch.rand((N, 6), device=d.device, generator=g) * 2.4 - 1.2
        od, rd, td, _, infd = d.step(a)
        oi, ri, ti, _, infi = i.step(a)
        assert torch.equal(rd, ri) and torch.equal(td, ti) and torch.equal(od, oi), t
        assert torch.equal(infd["reward_components"]["lung"], infi["reward_components"]["lung"])
        dl_d, dl_i = infd["doses"]["lung"].cpu().numpy(), infi["doses"]["lung"].cpu().numpy()
        bound = np.array([lung_inc_bound(x, lib.V) for x in dl_d])
        assert np.all(np.abs(dl_i.astype(np.float64) - dl_d) <= bound), t
    assert torch.equal(d.dose(), i.dose())
    d.close()
    i.close()


@pytest.mark.parametrize("mode", MODES)
def test_env_beam_list_is_the_applied_beam(dev, mode):
    """rt_env_beam_list returns the beam each env applied on its last step:
    dose_after == clip(dose_before + fl32(beam * 0.1f), 0, 1) on its voxels
    and unchanged elsewhere (environment.py:107-110), count 0 after resets."""
    lib = assets.synthetic_library((64, 64, 64), 64, 0)
    N = 48
    env = _vec_env(N, lib, seed=3, step_mode=mode)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(4)
    _, _, cnt = env.beam_list()
    assert int(cnt.abs().sum()) == 0  # nothing applied yet
    V = lib.V
    for t in range(104):  # crosses the t = 100 truncation and its autoreset
        before = env.dose().reshape(N, V).cpu().numpy()
        a = torch.rand((N, 6), device=dev, generator=g) * 2.4 - 1.2
        _, _, _, _, infos = env.step(a)
        idx, w, cnt = env.beam_list()
        after = env.dose().reshape(N, V).cpu().numpy()
        stepped = infos["_reward_components"].cpu().numpy()
        idx, w, cnt = idx.cpu().numpy(), w.cpu().numpy(), cnt.cpu().numpy()
        if t % 13 != 0 and t < 99:
            continue
        for e in range(N):
            if not stepped[e]:
                assert cnt[e] == 0 and not after[e].any()
                continue
            assert 0 < cnt[e] <= idx.shape[1] or cnt[e] == 0
            beam = np.zeros(V, np.float32)
            for i in range(cnt[e]):
                beam[idx[e, i]] = np.float32(beam[idx[e, i]] + w[e, i])
            want = np.clip(before[e] + beam * np.float32(0.1), np.float32(0), np.float32(1))
            np.testing.assert_array_equal(after[e].view(np.uint32), want.view(np.uint32), err_msg=f"t {t} env {e}")
    env.close()


def test_reset_seed_rekeys_tumour_stream(dev):
    """reset(seed=s) (rt_env_reseed): the tumours drawn afterwards are the
    Philox draws of key s from draw index 0 (tests/rt_rng.py), whatever the
    handle drew before -- a resumed run does not replay iteration 1's tumours
    and a given seed reproduces its sequence."""
    import rt_rng

    lib = assets.synthetic_library((64, 64, 64), 1000, 0)
    N = 64
    env = _vec_env(N, lib, seed=5)
    env.reset()
    env.reset()  # two draws on key 5
    first = env.get_state()[2].cpu().numpy()
    np.testing.assert_array_equal(first, [rt_rng.tumour_draw(5, e, 1, 1000) for e in range(N)])
    env.reset(seed=77)
    a = env.get_state()[2].cpu().numpy()
    np.testing.assert_array_equal(a, [rt_rng.tumour_draw(77, e, 0, 1000) for e in range(N)])
    env.reset()
    env.reset(seed=77)
    np.testing.assert_array_equal(env.get_state()[2].cpu().numpy(), a)
    env.close()


_LDS_ORDER = r"""
import sys
sys.path.insert(0, {repo!r})
import _rtpkg
import numpy as np, torch
from ppo_radiotherapy_amd import assets
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv
small = assets.synthetic_library((32, 32, 32), 8, 0)
ref = assets.synthetic_library((64, 64, 64), 8, 0)
# one 2400-voxel tumour: k_finish needs > 64 KiB of dynamic LDS on this handle
big = np.sort(np.random.default_rng(0).choice(64 ** 3, 2400, replace=False)).astype(np.int32)
vox = np.concatenate([ref.voxels, big])
off = np.concatenate([ref.offsets, [ref.offsets[-1] + big.size]])
lib = assets.TumourLibrary(shape=ref.shape, lungs=ref.lungs, names=ref.names + ["big"], voxels=vox, offsets=off)
for mode in ("dense", "incremental"):
    for L, ids in ((small, None), (lib, [8] * 16)):
        env = RadiotherapyVecEnv(16, visionless=True, library=L, seed=1, step_mode=mode)
        env.reset(options=None if ids is None else {{"tumour_ids": ids}})
        for t in range(3):
            env.step(torch.zeros((16, 6), device="cuda"))
        torch.cuda.synchronize()
        env.close()
print("lds-order ok")
"""


def test_small_then_large_lds_handle_in_one_process(dev):
    """a handle whose k_finish needs <= 64 KiB of LDS created first
    must not stop a later handle that needs more from launching (the dynamic-LDS
    limit is raised per kernel on first use).  Fresh process: the first launch
    of each kernel in it is the small handle's."""
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _LDS_ORDER.format(repo=repo)], capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0 and "lds-order ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
