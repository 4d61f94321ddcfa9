#!/usr/bin/env python3
"""Calibrate the CPU-baseline port (oracle/numpy_env.py) against the REAL
reference in the build container (within +-15 % of the
reference's steps/s on one core, same actions).

Runs only here (/root/reference is not on the GPU box).  Imports the
reference's environment.py read-only with tools/gen_golden.py's stand-ins for
the offline-absent gymnasium / SB3 / torchsummary, and times both on one
pinned core with the BASELINE.md §3 config C1 stream: reference grid and
tumour library, np.random.seed(1) tumour draws (environment.py:90, reset reads
the tumour file like the reference), actions default_rng(0).uniform(-1, 1,
(n, 6)).astype(float32), autoreset on done.  Every timing is a FRESH process
(the reference's cost depends on the allocator state of the process: in a
fresh one ~3 of its ~15 full-volume temporaries per step land on newly
faulted pages), alternating reference / port; also reported: minor page
faults per step.

    python tools/calibrate_cpu.py [--seconds 6 --rounds 3 --cpu 2]
prints one JSON object (committed as profiles/r03/cpu_calibration.json).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tools"), os.path.join(REPO, "oracle"), REPO]


def time_reference(ref, seconds):
    import gen_golden

    gen_golden.install_stubs()
    sys.dont_write_bytecode = True
    if ref not in sys.path:
        sys.path.insert(0, ref)
    with gen_golden.cwd(ref):
        import environment

        np.random.seed(1)
        env = environment.RadiotherapyEnv(visionless=True)
        rng = np.random.default_rng(0)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for a in rng.uniform(-1, 1, (64, 6)).astype(np.float32):
                done = env.step(a)[2]
                n += 1
                if done:
                    env.reset()
        return n / (time.perf_counter() - t0)


def time_port(seconds):
    import _rtpkg  # noqa: F401
    from numpy_env import NumpyEnv
    from ppo_radiotherapy_amd import assets

    lib = assets.reference_library()
    np.random.seed(1)
    draw = lambda: int(np.random.choice(lib.n_tumours))  # noqa: E731
    env = NumpyEnv(lib.lungs, lib.tumour_dense(draw()))
    env.reset()
    rng = np.random.default_rng(0)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for a in rng.uniform(-1, 1, (64, 6)).astype(np.float32):
            done = env.step(a)[-1]
            n += 1
            if done:
                env.reset(lib.tumour_dense(draw()))
    return n / (time.perf_counter() - t0)


def main():
    import resource
    import subprocess

    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--cpu", type=int, default=2)
    ap.add_argument("--one", choices=["reference", "port"], help="(child) time one kind in this process")
    ap.add_argument("--malloc", choices=["default", "pinned"], default="default",
                    help="pinned: mallopt(M_MMAP_THRESHOLD 32 MiB, M_TRIM_THRESHOLD 64 MiB) before anything runs, "
                         "so no full-volume temporary lands on freshly faulted pages (both kinds alike)")
    a = ap.parse_args()
    os.sched_setaffinity(0, {a.cpu})
    if a.one and a.malloc == "pinned":
        import ctypes

        libc = ctypes.CDLL("libc.so.6")
        assert libc.mallopt(-3, 32 << 20) == 1 and libc.mallopt(-1, 64 << 20) == 1
    if a.one:
        f0 = resource.getrusage(resource.RUSAGE_SELF).ru_minflt
        n0 = 0
        sps = time_reference(a.ref, a.seconds) if a.one == "reference" else time_port(a.seconds)
        faults = resource.getrusage(resource.RUSAGE_SELF).ru_minflt - f0
        print(json.dumps({"steps_per_s": sps, "faults_per_step": faults / max(sps * a.seconds, 1) + n0}))
        return
    res = {"reference": [], "port": []}
    for _ in range(a.rounds):
        for kind in ("reference", "port"):
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--one", kind, "--seconds", str(a.seconds),
                                  "--cpu", str(a.cpu), "--ref", a.ref, "--malloc", a.malloc],
                                 capture_output=True, text=True, check=True)
            res[kind].append(json.loads(out.stdout.strip().splitlines()[-1]))
    r = float(np.median([x["steps_per_s"] for x in res["reference"]]))
    p = float(np.median([x["steps_per_s"] for x in res["port"]]))
    print(json.dumps({"reference": res["reference"], "port": res["port"], "reference_median": r,
                      "port_median": p, "port_over_reference": p / r, "within_15pct": abs(p / r - 1) <= 0.15,
                      "cpu": a.cpu, "seconds_per_run": a.seconds, "process": "fresh per run", "malloc": a.malloc,
                      "config": "C1: reference grid + tumours, np.random.seed(1), default_rng(0) actions"}))


if __name__ == "__main__":
    main()
