"""Is the pipelined dense rollout host-bound?  The driver's value window
(20 rollout steps in one rt_env_rollout_policy call) is timed plainly, then
behind a gate: a one-block rt_probe_stream over a large buffer holds the
caller's stream while the host enqueues the whole call, so the window's GPU
time (HIP events from the gate's end to the call's end) carries no host
enqueue.  Same setup as bench.py (configs[1], staggered phases).

    python tools/r06/host_bound_probe.py [steps] [reps]
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import _rtpkg  # noqa: E402,F401
import bench  # noqa: E402
from ppo_radiotherapy_amd import _lib, assets  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    sys.argv = [sys.argv[0], "--no-cpu", "--no-c3d"]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    grid = (a.grid,) * 3
    lib = assets.synthetic_library(grid, 1000, 0)
    env = RadiotherapyVecEnv(a.envs, visionless=True, library=lib, device=dev, seed=a.seed, env_id_base=0)
    env.set_rollout_groups(2)
    torch.manual_seed(a.seed)
    agent = PPO((9,), (6,), 64).to(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(a.seed * 1000)
    tr = PPOTrainer(bench.trainer_cfg(a), env, agent, dev, 0, 1, gen)
    tr.reset()
    bench.stagger_phases(tr, env, dev)
    bench.run_steps(tr, 10)
    torch.cuda.synchronize()
    L = _lib.load()
    gate_buf = torch.zeros(60 << 20, device=dev)  # 240 MB read by one block: several ms
    sink = torch.zeros(4, device=dev)
    plain, gated, host_enq, gate_ms = [], [], [], []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        bench.run_steps(tr, K)
        torch.cuda.synchronize()
        plain.append((time.perf_counter() - t0) * 1e3 / K)
        # gated
        e_g0, e0, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
        torch.cuda.synchronize()
        e_g0.record()
        _lib.check(L.rt_probe_stream(gate_buf.data_ptr(), sink.data_ptr(), gate_buf.numel(), 0, 1,
                                     _lib.stream_handle()), "gate")
        e0.record()
        h0 = time.perf_counter()
        bench.run_steps(tr, K)
        host_enq.append((time.perf_counter() - h0) * 1e3)
        e1.record()
        torch.cuda.synchronize()
        gate_ms.append(e_g0.elapsed_time(e0))
        gated.append(e0.elapsed_time(e1) / K)
    med = lambda v: sorted(v)[len(v) // 2]
    print(f"steps {K} reps {reps}")
    print(f"plain  ms/step median {med(plain):.4f}  all {[round(x, 4) for x in plain]}")
    print(f"gated  ms/step median {med(gated):.4f}  all {[round(x, 4) for x in gated]}")
    print(f"host enqueue ms per call {[round(x, 3) for x in host_enq]}  gate ms {[round(x, 3) for x in gate_ms]}")
    print("valid: host enqueue < gate" if max(host_enq) < min(gate_ms) else "INVALID: the gate ended before the enqueue")


if __name__ == "__main__":
    main()
