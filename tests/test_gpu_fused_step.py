"""rt_env_step_policy (the policy fused into the env step: one launch per step
in incremental mode) produces the bits of rt_policy_sample + rt_env_step:
rollout storage, rewards, infos, observations, dose volumes and poses, across
episode ends (NEXT_STEP autoreset) and a block tail (N not a multiple of 16)."""
import os
import sys
from types import SimpleNamespace

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _cfg(fused_env_step):
    return SimpleNamespace(num_steps=32, num_minibatches=4, update_epochs=1, learning_rate=3e-4, anneal_lr=False,
                           gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                           vf_coef=0.5, max_grad_norm=0.5, seed=3, fused_env_step=fused_env_step)


def _trainer(mode, fused, lib, n):
    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    dev = torch.device("cuda")
    env = RadiotherapyVecEnv(n, visionless=True, library=lib, device=dev, seed=11, step_mode=mode)
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).to(dev)
    with torch.no_grad():
        agent.actor_logstd.fill_(0.3)  # wide actions: cone clamps, translation overshoot, beams missing the box
    tr = PPOTrainer(_cfg(fused), env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
    tr.reset()
    return tr


@pytest.mark.parametrize("mode", ["incremental", "dense"])
def test_fused_step_is_bitwise_the_two_call_step(mode):
    from ppo_radiotherapy_amd import assets

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    lib = assets.synthetic_library((40, 36, 44), 60, 2)
    n = 1000
    a = _trainer(mode, True, lib, n)
    b = _trainer(mode, False, lib, n)
    assert a.fused_env_step and not b.fused_env_step
    T = a.T
    ended = 0
    for it in range(5):  # 160 steps: every env passes max_time_steps = 100
        for t in range(T):
            a.rollout_step(t)
            b.rollout_step(t)
        torch.cuda.synchronize()
        for name in ("obs", "dones", "actions", "logprobs", "values", "rewards", "infos"):
            x, y = getattr(a, name), getattr(b, name)
            assert torch.equal(x.view(torch.int32), y.view(torch.int32)), f"{name} differs in iteration {it}"
        assert torch.equal(a.env.obs, b.env.obs) and torch.equal(a.env.terminated, b.env.terminated)
        pa, ta, ua = a.env.get_state()
        pb, tb, ub = b.env.get_state()
        assert torch.equal(pa, pb) and torch.equal(ta, tb) and torch.equal(ua, ub)
        assert torch.equal(a.env.dose(), b.env.dose())
        ended += int(a.dones.sum().item())
    assert ended >= n  # every env's first episode ended inside the compared steps
    a.env.close()
    b.env.close()
