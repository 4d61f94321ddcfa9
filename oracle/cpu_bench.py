"""CPU baseline timer for bench.py -- TEST/MEASUREMENT INFRASTRUCTURE ONLY.

Times the reference's single-env visionless step (environment.py:193-243) on
the host cores, on the same workload as the GPU bench:
the synthetic 64^3 library, U(-1,1) f32 actions from default_rng, autoreset
on done.  Two restatements:
  numpy  oracle/numpy_env.py -- op-for-op NumPy (dense volumes, Python-loop
         raster, scipy Rotation): tracks the reference's own cost per step
  c      oracle/rt_oracle.c  -- scalar C with the same dense passes
Each is timed on one core and on P cores (one pinned process per core,
aggregate steps/s).  Runs in its own process, started by bench.py as a child
so the GPU process never forks workers.

    python oracle/cpu_bench.py --grid 64 --seconds 10 --procs 8 --kinds numpy,c
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

    return assets.synthetic_library((grid,) * 3, 1000, 0)


def _worker(kind, grid, seconds, seed, cpu, q):
    if cpu is not None:
        try:
            os.sched_setaffinity(0, {cpu})
        except OSError:
            pass
    lib = _library(grid)
    if kind == "numpy":
        from numpy_env import NumpyEnv
        env = NumpyEnv(lib.lungs, lib.tumour_dense(seed % lib.n_tumours))
    else:
        from oracle import OracleEnv
        env = OracleEnv(lib.lungs, lib.tumour_dense(seed % lib.n_tumours))
    rng = np.random.default_rng(seed)
    env.reset()
    n, t0 = 0, time.perf_counter()
    while True:
        a = rng.uniform(-1, 1, 6).astype(np.float32)
        done = env.step(a)[-1]
        n += 1
        if done:
            env.reset(lib.tumour_dense(int(rng.integers(lib.n_tumours))))
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    q.put((n, dt))


def run(kind, grid, seconds, procs):
    """Aggregate steps/s of `procs` pinned single-env processes."""
    ctx = mp.get_context("fork")
    cpus = sorted(os.sched_getaffinity(0))
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(kind, grid, seconds, i, cpus[i % len(cpus)] if procs > 1 else None, q))
          for i in range(procs)]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=64)
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--procs", type=int, default=0, help="0 = min(available cores, 16)")
    ap.add_argument("--kinds", default="numpy,c")
    a = ap.parse_args()
    avail = len(os.sched_getaffinity(0))
    procs = a.procs or min(avail, 16)
    out = {"cpu_model": cpu_model(), "cores_available": avail}
    for kind in a.kinds.split(","):
        out[kind] = {"one_core": run(kind, a.grid, a.seconds, 1)}
        if procs > 1:
            out[kind]["all_cores"] = run(kind, a.grid, a.seconds, procs)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
