"""PMC companion of probe_steady.py: one env group (grid k_dense), a
staggered window and a phase-locked window of 32 steps each.  k_dense
dispatch order: 1 (reset) + 16 + 200 (stagger: reset call + step) +
32 staggered + 17 (lock: reset + 16) + 32 locked = 298."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import _rtpkg  # noqa
import torch
from types import SimpleNamespace
from ppo_radiotherapy_amd import assets
from ppo_radiotherapy_amd.networks import PPO
from ppo_radiotherapy_amd.ppo import PPOTrainer
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv
import bench

dev = torch.device("cuda")
lib = assets.synthetic_library((64, 64, 64), 1000, 0)
N = 4096
env = RadiotherapyVecEnv(N, library=lib, device=dev, seed=1, step_mode="dense")
env.set_rollout_groups(1)
torch.manual_seed(1)
agent = PPO((9,), (6,), 64).to(dev)
cfg = SimpleNamespace(num_steps=64, num_minibatches=8, update_epochs=10, learning_rate=3e-4, anneal_lr=False,
                      gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                      vf_coef=0.5, max_grad_norm=0.5, micro_batch=0)
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
bench.run_steps(tr, 16)
e_idx = torch.arange(N, device=dev)
for k in range(100):
    env.reset(options={"mask": (e_idx % 100) == k})
    tr.rollout_steps(k % 64, 1)
bench.run_steps(tr, 32)
env.reset()
bench.run_steps(tr, 16)
bench.run_steps(tr, 32)
torch.cuda.synchronize()
env.close()
print("done")
