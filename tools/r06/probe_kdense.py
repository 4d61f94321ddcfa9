"""k_dense alone on the chip (one env group: the stepwise launches), 4096
envs x 64^3 on staggered episode phases, 30 rollout steps -- the
rocprofv3 / PMC subject for the lung-stream kernel (round 6)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
env.set_rollout_groups(int(os.environ.get("GROUPS", "1")))
torch.manual_seed(1)
agent = PPO((9,), (6,), 64).to(dev)
cfg = bench.trainer_cfg(bench.argparse.Namespace(num_steps=64, num_minibatches=8, update_epochs=10, micro_batch=0,
                                                 update_precision="f32", vision=False))
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
bench.stagger_phases(tr, env, dev)
bench.run_steps(tr, 30)
torch.cuda.synchronize()
env.close()
print("done", flush=True)
