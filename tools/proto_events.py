"""Prototype: cost of the per-step timing events and of the null stream on the
rollout (dense and incremental), 4096 envs at 64^3."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

import proto_split as ps  # noqa: E402
import bench  # noqa: E402
from ppo_radiotherapy_amd import assets  # noqa: E402


def timed(tr, K, timing, stream):
    if timing:
        tr.env.kernel_timing(K)
    torch.cuda.synchronize()
    ctx = torch.cuda.stream(stream) if stream is not None else torch.cuda.stream(torch.cuda.current_stream())
    with ctx:
        for i in range(8):
            tr.rollout_step(i % tr.T)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(K):
            tr.rollout_step(i % tr.T)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    if timing:
        tr.env.kernel_timing_read()
        tr.env.kernel_timing(0)
    return tr.N * K / dt


def main():
    sys.argv = [sys.argv[0]]
    a = bench.parse()
    dev = torch.device("cuda", 0)
    lib = assets.synthetic_library((64,) * 3, 1000, 0)
    out = {}
    for mode in ("dense", "incremental"):
        tr = ps.make(4096, 0, lib, dev, a, mode)
        side = torch.cuda.Stream()
        for name, timing, st in (("null", False, None), ("null_timing", True, None),
                                 ("side", False, side), ("side_timing", True, side), ("null2", False, None)):
            out[f"{mode}_{name}"] = timed(tr, 64, timing, st)
        tr.env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
