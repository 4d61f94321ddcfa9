"""Micro-benchmark of the PPO update phase under different BLAS backends."""
import os
import sys
import time
from types import SimpleNamespace

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import _rtpkg  # noqa
from fake_env import FakeVecEnv, torch_gae  # noqa
from ppo_radiotherapy_amd.networks import PPO  # noqa
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa


def run(backend):
    if backend:
        torch.backends.cuda.preferred_blas_library(backend)
    dev = torch.device("cuda")
    cfg = SimpleNamespace(num_steps=64, num_minibatches=8, update_epochs=10, learning_rate=3e-4, anneal_lr=False,
                          gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                          vf_coef=0.5, max_grad_norm=0.5)
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).to(dev)
    env = FakeVecEnv(4096)
    tr = PPOTrainer(cfg, env, agent, dev, generator=torch.Generator(device=dev).manual_seed(0))
    tr.obs.normal_()
    tr.actions.normal_()
    tr.advantages.normal_()
    tr.returns.normal_()
    tr.values.normal_()
    tr.update()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 0
    for _ in range(3):
        n += tr.update()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"backend={backend or 'default'} updates/s={n / dt:.1f} ms/update={1000 * dt / n:.3f}", flush=True)


if __name__ == "__main__":
    run(sys.argv[1] if len(sys.argv) > 1 else None)
