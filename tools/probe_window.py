"""Does a rollout call pay a fixed cost? bench.py's workload (4096 envs x 64^3,
dense, 2 pipelined env groups, the trainer's rollout call), windows of K
steps timed like bench.py's value pass (synchronize, perf_counter, one or more
rollout calls, synchronize), K = 20 / 64 / 128, each both right after a PPO
update (as bench.py's value pass is) and after another rollout window.  A
one-block rt_probe_stream launch marks every window for a kernel trace
(tools/steady_trace.py reads it).  Prints one JSON line per window."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import _rtpkg  # noqa: E402,F401
import torch  # noqa: E402

import bench  # noqa: E402
from ppo_radiotherapy_amd import _lib, assets  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
lib = assets.synthetic_library((64, 64, 64), 1000, 0)
env = RadiotherapyVecEnv(4096, library=lib, device=dev, seed=1)
env.set_rollout_groups(int(os.environ.get("GROUPS", "2")))
torch.manual_seed(1)
agent = PPO((9,), (6,), 64).to(dev)
cfg = bench.trainer_cfg(bench.argparse.Namespace(num_steps=64, num_minibatches=8, update_epochs=10, micro_batch=0))
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
L = _lib.load()
mark_buf = torch.zeros(4, device=dev)


def mark():
    _lib.check(L.rt_probe_stream(mark_buf.data_ptr(), mark_buf.data_ptr(), 4, 0, 1, _lib.stream_handle()), "mark")


bench.run_steps(tr, 16)
tr.compute_gae()
tr.update()
torch.cuda.synchronize()
for rep in range(2):
    for K in (20, 64, 128):
        for after in ("update", "rollout"):
            if after == "update":
                tr.compute_gae()
                tr.update()
            else:
                bench.run_steps(tr, 16)
            mark()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            bench.run_steps(tr, K)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps({"rep": rep, "K": K, "after": after, "ms": 1000 * dt, "ms_per_step": 1000 * dt / K,
                              "env_steps_per_s": 4096 * K / dt}), flush=True)
mark()
env.close()
