"""Prototype: does splitting the rollout's envs into independent halves on two
HIP streams overlap the latency-bound kernels (policy, k_beam, k_finish) of
one half with the HBM-bound k_dense of the other?  Compares K rollout steps of
one 4096-env trainer against two 2048-env trainers on two streams.

    python tools/proto_split.py [--parts 2]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

import _rtpkg  # noqa: E402,F401
from ppo_radiotherapy_amd import assets  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: E402

sys.path.insert(0, REPO)
import bench  # noqa: E402


def make(n, base, lib, dev, a, mode):
    env = RadiotherapyVecEnv(n, visionless=True, library=lib, device=dev, seed=1, env_id_base=base, step_mode=mode)
    torch.manual_seed(1)
    agent = PPO((9,), (6,), 64).to(dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000)
    tr = PPOTrainer(bench.trainer_cfg(a), env, agent, dev, 0, 1, gen)
    tr.reset()
    return tr


def run(trs, streams, K, T):
    main = torch.cuda.current_stream()
    for s in streams:
        s.wait_stream(main)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(K):
        for tr, s in zip(trs, streams):
            with torch.cuda.stream(s):
                tr.rollout_step(i % T)
    for s in streams:
        main.wait_stream(s)
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--parts", type=int, default=2)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--mode", default="dense")
    a0 = ap.parse_args()
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    lib = assets.synthetic_library((64,) * 3, 1000, 0)
    N, K = 4096, a0.steps
    res = {}
    one = make(N, 0, lib, dev, a, a0.mode)
    s1 = [torch.cuda.Stream()]
    run([one], s1, 16, one.T)
    res["one"] = N * K / run([one], s1, K, one.T)
    one.env.close()
    del one
    for P in (2, 4):
        n = N // P
        trs = [make(n, p * n, lib, dev, a, a0.mode) for p in range(P)]
        ss = [torch.cuda.Stream() for _ in range(P)]
        run(trs, ss, 16, trs[0].T)
        res[f"split{P}"] = N * K / run(trs, ss, K, trs[0].T)
        res[f"split{P}_serial_stream"] = N * K / run(trs, [ss[0]] * P, K, trs[0].T)
        for tr in trs:
            tr.env.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
