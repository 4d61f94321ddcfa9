"""Pipelined dense rollout (bench workload, 4096 envs x 64^3): wall ms per
step with and without the library's per-kernel timing events, alternating
passes.  python tools/probe_timing_cost.py [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import _rtpkg  # noqa: E402,F401
import torch  # noqa: E402

from ppo_radiotherapy_amd import assets  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
lib = assets.synthetic_library((64, 64, 64), 1000, 0)
env = RadiotherapyVecEnv(4096, visionless=True, library=lib, device=dev, seed=1)
env.set_rollout_groups(2)
torch.manual_seed(1)
agent = PPO((9,), (6,), 64).to(dev)
cfg = bench.trainer_cfg(type("A", (), dict(num_steps=64, num_minibatches=8, update_epochs=10, micro_batch=0))())
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
bench.run_steps(tr, 16)
torch.cuda.synchronize()
res = {"timing_on": [], "timing_off": []}
for rep in range(4):
    for mode in ("timing_on", "timing_off"):
        env.kernel_timing(2 * K if mode == "timing_on" else 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bench.run_steps(tr, K)
        torch.cuda.synchronize()
        res[mode].append(1000 * (time.perf_counter() - t0) / K)
        if mode == "timing_on":
            env.kernel_timing_read()
# host enqueue time of one 64-step rollout call (no sync) vs its GPU time
env.kernel_timing(0)
enq = []
for rep in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.run_steps(tr, K)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    enq.append((1000 * (t1 - t0) / K, 1000 * (t2 - t0) / K))
print("enqueue_ms_per_step, total_ms_per_step:", [(round(a, 4), round(b, 4)) for a, b in enq])
print({k: [round(x, 4) for x in v] for k, v in res.items()})
print({k: min(v) for k, v in res.items()})
