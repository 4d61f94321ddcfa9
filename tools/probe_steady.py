"""Where the steady-state step time goes (dense pipelined rollout, 4096 envs
x 64^3): phase-locked windows before / across the t = 100 reset wave and a
staggered window, per-kernel HIP-event times, 1 and 2 env groups."""
import json
import os
import sys
import time

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


def window(tr, env, K, label):
    env.kernel_timing(2 * K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.run_steps(tr, K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    kms, n = env.kernel_timing_read()
    env.kernel_timing(0)
    print(json.dumps({"label": label, "ms_per_step": 1000 * dt / K,
                      "kernels_ms_per_step": {k: round(v * n / K, 4) for k, v in kms.items()}}), flush=True)


def stagger(tr, env):
    e_idx = torch.arange(N, device=dev)
    for k in range(100):
        env.reset(options={"mask": (e_idx % 100) == k})
        tr.rollout_steps(k % 64, 1)


def lock(tr, env):
    env.reset()
    bench.run_steps(tr, 16)


for groups in (2, 1):
    env = RadiotherapyVecEnv(N, library=lib, device=dev, seed=1, step_mode="dense")
    env.set_rollout_groups(groups)
    torch.manual_seed(1)
    agent = PPO((9,), (6,), 64).to(dev)
    cfg = SimpleNamespace(num_steps=64, num_minibatches=8, update_epochs=10, learning_rate=3e-4, anneal_lr=False,
                          gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                          vf_coef=0.5, max_grad_norm=0.5, micro_batch=0)
    tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
    tr.reset()
    bench.run_steps(tr, 16)
    for rep in range(2):
        stagger(tr, env)
        window(tr, env, 64, f"g{groups} staggered rep{rep}")
        lock(tr, env)
        window(tr, env, 64, f"g{groups} locked t=16..80 rep{rep}")
        stagger(tr, env)
        window(tr, env, 64, f"g{groups} staggered-b rep{rep}")
    env.close()
