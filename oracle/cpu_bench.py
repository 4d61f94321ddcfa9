"""CPU baseline timer for bench.py -- TEST/MEASUREMENT INFRASTRUCTURE ONLY.

Times the reference's single-env visionless step (environment.py:193-243) on
the host cores.  Default workload = BASELINE.md §3 / SURVEY §8d config C1:
the reference grid 67x43x70 (data/lungs.npy) and the reference's 1000
tumours, the tumour of every episode drawn with `np.random.seed(1)` +
`np.random.choice` (environment.py:90), actions
`default_rng(0).uniform(-1, 1, (n, 6)).astype(float32)`, autoreset on done.
(`--grid 64` times the GPU bench's 64^3 synthetic workload instead.)
Two restatements:
  numpy  oracle/numpy_env.py -- op-for-op NumPy (dense volumes, Python-loop
         raster, scipy Rotation): tracks the reference's own cost per step
  c      oracle/rt_oracle.c  -- scalar C with the same dense passes
Each is timed on one core (the process pinned to one CPU, like `taskset -c
0`) and on P cores (one pinned process per core, aggregate steps/s; process
i uses np.random.seed(1 + i) and default_rng(i)).  Runs in its own process,
started by bench.py as a child so the GPU process never forks workers.

    python oracle/cpu_bench.py --seconds 10 --procs 16 --kinds numpy,c
prints one JSON object.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)


def _library(grid):
    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd import assets

    if grid == 0:  # config C1: the reference's own assets
        return assets.reference_library()
    return assets.synthetic_library((grid,) * 3, 1000, 0)


def pin_allocator():
    """Fixed glibc allocator thresholds (mmap 32 MiB, trim 64 MiB) before any
    volume is allocated: every full-volume temporary is then served from the
    heap without fresh page faults.  This is the regime the reference's
    published 294 steps/s/core and its calibration here run
    in (tools/calibrate_cpu.py --malloc pinned: reference 291, port 281
    steps/s); a fresh default-allocator reference process pays ~650 minor
    faults per step and runs ~185 steps/s, so the pinned baseline is the
    FASTER CPU reference."""
    import ctypes

    try:
        libc = ctypes.CDLL("libc.so.6")
        return bool(libc.mallopt(-3, 32 << 20) == 1 and libc.mallopt(-1, 64 << 20) == 1)
    except OSError:
        return False


def _worker(kind, grid, seconds, seed, cpu, q):
    pin_allocator()
    if cpu is not None:
        try:
            os.sched_setaffinity(0, {cpu})
        except OSError:
            pass
    lib = _library(grid)
    np.random.seed(1 + seed)                  # environment.py:90's global stream
    draw = lambda: int(np.random.choice(lib.n_tumours))  # noqa: E731
    if kind == "numpy":
        from numpy_env import NumpyEnv
        env = NumpyEnv(lib.lungs, lib.tumour_dense(draw()))
    else:
        from oracle import OracleEnv
        env = OracleEnv(lib.lungs, lib.tumour_dense(draw()))
    rng = np.random.default_rng(seed)
    env.reset()
    n, t0 = 0, time.perf_counter()
    while True:
        acts = rng.uniform(-1, 1, (256, 6)).astype(np.float32)  # the same stream as one (n, 6) draw
        for a in acts:
            done = env.step(a)[-1]
            n += 1
            if done:
                env.reset(lib.tumour_dense(draw()))
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    q.put((n, dt))


def run(kind, grid, seconds, procs):
    """Aggregate steps/s of `procs` pinned single-env processes."""
    ctx = mp.get_context("fork")
    cpus = sorted(os.sched_getaffinity(0))
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(kind, grid, seconds, i, cpus[i % len(cpus)], q)) for i in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    return {"steps": int(sum(n for n, _ in res)), "value": float(sum(n / dt for n, dt in res)),
            "seconds": float(max(dt for _, dt in res)), "cores": procs}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


# The GPU box grants one GPU's job a 16-core CPU share (gpurun pool rule; the
# host shows all of its cores to os.sched_getaffinity): the all-cores leg
# uses at most that many pinned processes.
CORE_SHARE = 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=0, help="0 = config C1 (reference 67x43x70 grid and tumours)")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--procs", type=int, default=0, help=f"0 = min(available cores, {CORE_SHARE})")
    ap.add_argument("--kinds", default="numpy,c")
    a = ap.parse_args()
    avail = len(os.sched_getaffinity(0))
    procs = a.procs or min(avail, CORE_SHARE)
    out = {"cpu_model": cpu_model(), "cores_available": avail,
           "allocator": "glibc mallopt pinned (mmap 32 MiB / trim 64 MiB): no page faults on full-volume temporaries",
           "config": ("C1: reference 67x43x70 lungs + 1000 reference tumours, np.random.seed(1) tumour draws, "
                      "default_rng(0) U(-1,1) f32 actions, autoreset" if a.grid == 0 else
                      f"{a.grid}^3 synthetic library, U(-1,1) f32 actions, autoreset"),
           "cores_cap": (f"all-cores leg: {procs} pinned processes (--procs)" if a.procs else
                         f"all-cores leg: {procs} pinned processes = the box's {CORE_SHARE}-core share per GPU "
                         f"of {avail} visible" if procs < avail else f"all {avail} available cores")}
    for kind in a.kinds.split(","):
        out[kind] = {"one_core": run(kind, a.grid, a.seconds, 1)}
        if procs > 1:
            out[kind]["all_cores"] = run(kind, a.grid, a.seconds, procs)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
