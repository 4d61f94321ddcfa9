"""PMC companion of bench.py's dense pipelined rollout (4096 envs x 64^3, two
env groups, k_dense over 2048 envs per launch), in bench.py's order:
200 launches of the stagger pre-roll (100 one-step calls; every env's episode
clock offset by e % 100), 10 (5 warm steps), 40 (a 20-step window, the
`value` shape) and 128 (a 64-step window, the steady-state shape).  With the
phases staggered ~1 % of the envs reset every step in both windows, each
reset zeroing its dose row inside k_dense.
tools/dense_pmc_segments.py splits the counter rows by that order."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import _rtpkg  # noqa: E402,F401
import torch  # noqa: E402

import bench  # noqa: E402
from ppo_radiotherapy_amd import assets  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: E402

dev = torch.device("cuda", 0)
lib = assets.synthetic_library((64, 64, 64), 1000, 0)
N = 4096
env = RadiotherapyVecEnv(N, library=lib, device=dev, seed=1)
env.set_rollout_groups(2)
torch.manual_seed(1)
agent = PPO((9,), (6,), 64).to(dev)
cfg = bench.trainer_cfg(bench.argparse.Namespace(num_steps=64, num_minibatches=8, update_epochs=10, micro_batch=0,
                                                 update_precision="f32", vision=False))
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
bench.stagger_phases(tr, env, dev)
bench.run_steps(tr, 5)
bench.run_steps(tr, 20)
bench.run_steps(tr, 64)
torch.cuda.synchronize()
env.close()
print("done", flush=True)
