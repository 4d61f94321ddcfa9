"""Why does the first timed 20-step window of the driver's bench command
(`bench.py --gpus 1 --steps 20 --warmup 5`) run slower than the identical
second one?  Reproduces the round-3 bench sequence -- reset, 2 rollout steps,
GAE + update, 3 rollout steps, then back-to-back 20-step windows (the second
with the library's timing events, as bench.py's instrumented pass) -- and a
few controls: a window right after an update, one after an idle gap, and the
same windows with staggered episode phases.  A one-block rt_probe_stream
launch marks every window, so a rocprofv3 kernel trace of this script can be
cut per window (tools/window_kernels.py).  One JSON line per window."""
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
env.set_rollout_groups(2)
torch.manual_seed(1)
agent = PPO((9,), (6,), 64).to(dev)
cfg = bench.trainer_cfg(bench.argparse.Namespace(num_steps=64, num_minibatches=8, update_epochs=10, micro_batch=0,
                                                 update_precision="f32", vision=False))
tr = PPOTrainer(cfg, env, agent, dev, 0, 1, torch.Generator(device=dev).manual_seed(1))
tr.reset()
L = _lib.load()
mark_buf = torch.zeros(4, device=dev)
seq = [0]


def mark():
    _lib.check(L.rt_probe_stream(mark_buf.data_ptr(), mark_buf.data_ptr(), 4, 0, 1, _lib.stream_handle()), "mark")


def window(tag, K=20, events=False):
    if events:
        env.kernel_timing(2 * K)
    mark()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bench.run_steps(tr, K)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if events:
        env.kernel_timing(0)
    seq[0] += 1
    print(json.dumps({"seq": seq[0], "tag": tag, "K": K, "ms_per_step": 1000 * dt / K,
                      "env_steps_per_s": 4096 * K / dt}), flush=True)


def update():
    tr.compute_gae()
    tr.update()


# the round-3 driver sequence
bench.run_steps(tr, 2)
update()
bench.run_steps(tr, 3)
torch.cuda.synchronize()
window("A_first_after_warmup")
window("B_second_events", events=True)
window("C_third")
window("D_fourth")
# right after an update, then again
update()
torch.cuda.synchronize()
window("E_right_after_update")
window("F_next")
update()
bench.run_steps(tr, 3)
torch.cuda.synchronize()
window("G_3steps_after_update")
window("H_next")
# after an idle gap (clock ramp?)
time.sleep(0.5)
window("I_after_0.5s_idle")
window("J_next")
# staggered episode phases (bench.py's pre-roll), then the same pattern
e_idx = torch.arange(4096, device=dev)
for k in range(100):
    env.reset(options={"mask": (e_idx % 100) == k})
    tr.rollout_steps(k % tr.T, 1)
update()
bench.run_steps(tr, 3)
torch.cuda.synchronize()
window("S1_staggered_after_update")
window("S2_staggered_events", events=True)
window("S3_staggered")
window("S4_staggered_64", K=64)
mark()
torch.cuda.synchronize()
env.close()
