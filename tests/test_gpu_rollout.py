"""rt_env_rollout_policy produces the bits of stepwise rt_env_step_policy
launches: rollout storage, rewards, infos, observations, dose volumes and
poses, across episode ends (NEXT_STEP autoreset), a block tail (N not a
multiple of 16), runs that start mid-storage, and libraries whose largest
tumour's sum plan exceeds a wave's LDS region.  Incremental step mode: the
whole rollout as ONE persistent launch (one wave per env running its steps
back to back; plan slots in the global scratch row for 1000 and 12000 voxel
tumours).  Dense step mode: the stepwise launches of two to four env groups
pipelined over library streams, and the one-group variant (every launch on
the caller's stream)."""
import os
import sys
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _cfg(fused_rollout):
    return SimpleNamespace(num_steps=32, num_minibatches=4, update_epochs=1, learning_rate=3e-4, anneal_lr=False,
                           gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                           vf_coef=0.5, max_grad_norm=0.5, seed=3, fused_env_step=True, fused_rollout=fused_rollout)


def _trainer(fused_rollout, lib, n, step_mode="incremental"):
    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    dev = torch.device("cuda")
    env = RadiotherapyVecEnv(n, visionless=True, library=lib, device=dev, seed=11, step_mode=step_mode)
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).to(dev)
    with torch.no_grad():
        agent.actor_logstd.fill_(0.3)  # wide actions: cone clamps, translation overshoot, beams missing the box
    tr = PPOTrainer(_cfg(fused_rollout), env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
    tr.reset()
    return tr


def _with_big_tumour(lib, n_vox):
    """`lib` with its last tumour replaced by a box of n_vox voxels."""
    from ppo_radiotherapy_amd.assets import TumourLibrary

    D, H, W = lib.shape
    side = int(np.ceil(n_vox ** (1 / 3)))
    z0, y0, x0 = D // 2 - side // 2, H // 2 - side // 2, W // 2 - side // 2
    box = np.array([(z0 + i) * H * W + (y0 + j) * W + (x0 + k)
                    for i in range(side) for j in range(side) for k in range(side)][:n_vox], dtype=np.int32)
    box.sort()
    K = lib.n_tumours
    vox = np.concatenate([lib.voxels[:lib.offsets[K - 1]], box]).astype(np.int32)
    off = np.concatenate([lib.offsets[:K], [len(vox)]]).astype(np.int64)
    return TumourLibrary(lib.shape, lib.lungs, list(lib.names), vox, off)


def _compare(a, b, it):
    for name in ("obs", "dones", "actions", "logprobs", "values", "rewards", "infos"):
        x, y = getattr(a, name), getattr(b, name)
        assert torch.equal(x.view(torch.int32), y.view(torch.int32)), f"{name} differs in iteration {it}"
    assert torch.equal(a.env.obs, b.env.obs) and torch.equal(a.env.terminated, b.env.terminated)
    pa, ta, ua = a.env.get_state()
    pb, tb, ub = b.env.get_state()
    assert torch.equal(pa, pb) and torch.equal(ta, tb) and torch.equal(ua, ub)
    assert torch.equal(a.env.dose(), b.env.dose())


@pytest.mark.parametrize("step_mode,big,groups", [("incremental", 0, 0), ("incremental", 1000, 0),
                                                   ("incremental", 12000, 0), ("dense", 0, 2),
                                                   ("dense", 1000, 2), ("dense", 0, 3),
                                                   ("dense", 1000, 4), ("dense", 0, 1), ("dense", 12000, 2)])
def test_rollout_call_is_bitwise_the_stepwise_rollout(step_mode, big, groups):
    from ppo_radiotherapy_amd import assets

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    lib = assets.synthetic_library((40, 36, 44), 60, 2)
    if big:
        lib = _with_big_tumour(lib, big)
    n = 1000
    a = _trainer(True, lib, n, step_mode)
    b = _trainer(False, lib, n, step_mode)
    if step_mode == "dense":
        a.env.set_rollout_groups(groups)
    assert a.fused_rollout and not b.fused_rollout
    T = a.T
    # runs of storage rows per iteration: whole rollouts and split ones
    runs = [[(0, T)], [(0, 5), (5, T - 5)], [(0, 1), (1, 30), (31, 1)], [(0, T)], [(0, 17), (17, 15)]]
    ended = seen_big = 0
    for it, rr in enumerate(runs):  # 160 steps: every env passes max_time_steps = 100
        for first, count in rr:
            a.rollout_steps(first, count)
            b.rollout_steps(first, count)
        torch.cuda.synchronize()
        _compare(a, b, it)
        ended += int(a.dones.sum().item())
        seen_big += int(a.env.get_state()[2].eq(lib.n_tumours - 1).sum().item())
    assert ended >= n  # every env's first episode ended inside the compared steps
    assert a.fused_rollout  # the rollout call ran every run
    assert seen_big > 0  # some envs ran episodes on the largest tumour
    a.env.close()
    b.env.close()


def test_rollout_policy_rejects_vision_and_bad_groups():
    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd import _lib, assets
    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    lib = assets.synthetic_library((40, 36, 44), 20, 2)
    env = RadiotherapyVecEnv(64, visionless=True, library=lib, device="cuda", seed=1, step_mode="dense")
    tr = PPOTrainer(_cfg(True), env, PPO((9,), (6,), 64).cuda(), torch.device("cuda"), 0, 1)
    tr.reset()
    ro = tr._rollout_struct(0, 4)
    with pytest.raises(_lib.RtError, match="groups"):
        env.set_rollout_groups(5)
    with pytest.raises(_lib.RtError, match="groups"):
        env.set_rollout_groups(-1)
    with pytest.raises(_lib.RtError, match="groups"):
        env.set_rollout_groups(16)  # the round-5 dataflow value, removed (ABI 5)
    with pytest.raises(_lib.RtError, match="incremental"):
        env.set_rollout_groups(0)  # the persistent launch is the incremental mode's
    env.close()
    ienv = RadiotherapyVecEnv(64, visionless=True, library=lib, device="cuda", seed=1, step_mode="incremental")
    ienv.set_rollout_groups(0)
    with pytest.raises(_lib.RtError, match="incremental"):
        ienv.set_rollout_groups(2)
    ienv.close()
    venv = RadiotherapyVecEnv(4, visionless=False, library=lib, device="cuda", seed=1)
    with pytest.raises(_lib.RtError, match="visionless"):
        venv.rollout_policy(ro)
    venv.close()


@pytest.mark.parametrize("n,groups", [(1, 2), (17, 2), (33, 2), (70, 3), (5, 1), (33, 4)])
def test_small_handles_rollout_bitwise(n, groups):
    """Edge sizes of the dense rollout call: a single env, fewer envs than two
    16-env groups (the call falls back to one group), group boundaries off
    the block size -- each bitwise the stepwise launches over 128 steps (every env passes
    its t = 100 truncation autoreset)."""
    from ppo_radiotherapy_amd import assets

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    lib = assets.synthetic_library((40, 36, 44), 60, 2)
    a = _trainer(True, lib, n, "dense")
    b = _trainer(False, lib, n, "dense")
    a.env.set_rollout_groups(groups)
    T = a.T
    for it in range(4):
        a.rollout_steps(0, T)
        b.rollout_steps(0, T)
        torch.cuda.synchronize()
        _compare(a, b, it)
    assert a.fused_rollout
    a.env.close()
    b.env.close()
