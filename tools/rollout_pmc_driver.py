"""Runs the incremental-mode rollout (4096 envs, 64^3, persistent
k_rollout_policy launches of 64 steps) a few times -- a target for
rocprofv3 --pmc / --kernel-trace.  --stepwise runs the per-step fused launches."""
import os
import sys
from types import SimpleNamespace

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402

from ppo_radiotherapy_amd import assets  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: E402

dev = torch.device("cuda")
lib = assets.synthetic_library((64, 64, 64))
env = RadiotherapyVecEnv(4096, visionless=True, library=lib, device=dev, seed=1, step_mode="incremental")
cfg = SimpleNamespace(num_steps=64, num_minibatches=8, update_epochs=10, learning_rate=3e-4, anneal_lr=False,
                      gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                      vf_coef=0.5, max_grad_norm=0.5, seed=1, fused_rollout="--stepwise" not in sys.argv)
torch.manual_seed(0)
agent = PPO((9,), (6,), 64).to(dev)
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
for _ in range(4):
    tr.rollout()
torch.cuda.synchronize()
print("ok")
