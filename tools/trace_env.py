"""Phase timeline of one rollout step (policy + env kernels), per env.

Builds a traced copy of librtenv.so (-DRT_TRACE: s_memrealtime stamps at the
phase boundaries of k_policy_sample, k_beam and k_finish; csrc/rt_trace.h),
runs the fused-policy rollout for a few steps and prints, for the last step,
each phase's per-env duration (median / p90 / max, us) and each kernel's
start/end spread relative to the step's first stamp.

    python tools/trace_env.py [--mode incremental|dense] [--envs 4096] [--build-only]
                              [--pipelined [--stagger]]   (dense: the two-group rollout call)
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tools", "_trace", "librtenv_trace.so")
SLOTS, CAP = 16, 8192
PHASES = {  # name: (start slot, end slot)
    "policy": (0, 1), "policy.stage": (0, 9), "policy.mlp+sample": (9, 1), "beam.pose": (2, 3), "pose.loads": (2, 10), "pose.update": (10, 11), "pose.setup": (11, 3), "pose->march": (3, 12), "beam.march": (12, 4), "finish.gather": (5, 6),
    "finish.plan": (6, 7), "finish.tail": (7, 8), "policy->beam": (1, 2), "beam->finish": (4, 5),
    "step": (0, 8),
}


def build():
    sys.path.insert(0, os.path.join(REPO, "ppo-radiotherapy_amd"))
    import build as b
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cmd = [b.hipcc(), *b.HIPCC_FLAGS, "-shared", *b.EXTRA_FLAGS[b.SRC], "-DRT_TRACE", "-I", os.path.join(REPO, "include"),
           *b.SRCS, "-o", OUT]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="incremental")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=24)
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--two-call", action="store_true", help="rt_policy_sample + rt_env_step instead of the fused step")
    ap.add_argument("--pipelined", action="store_true",
                    help="dense mode: the pipelined two-group rollout call (rt_env_rollout_policy); stamps of the last step")
    ap.add_argument("--dump", default=None, help="also save the raw stamp table (us, [envs][16]) to this .npy")
    ap.add_argument("--stagger", action="store_true", help="staggered episode phases first (bench.stagger_phases)")
    ap.add_argument("--persistent", action="store_true",
                    help="the steps as one persistent k_rollout_policy launch (incremental); stamps of the last step")
    a = ap.parse_args()
    if a.build_only or not os.path.exists(OUT):
        build()
    if a.build_only:
        return
    import torch
    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd import _lib
    _lib.LIB_PATH = OUT
    L = _lib.load(build_if_missing=False)
    sys.argv = [sys.argv[0]]
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench
    import proto_split as ps
    from ppo_radiotherapy_amd import assets
    cfg = bench.parse()
    dev = torch.device("cuda", 0)
    lib = assets.synthetic_library((64,) * 3, 1000, 0)
    cfg.fused_env_step = not a.two_call
    tr = ps.make(a.envs, 0, lib, dev, cfg, a.mode)
    if a.stagger:
        bench.stagger_phases(tr, tr.env, dev)
    if a.pipelined:
        tr.fused_rollout = True
        tr.env.set_rollout_groups(2)
        tr.rollout_steps(0, min(a.steps, tr.T))
    elif a.persistent:
        tr.fused_rollout = True
        tr.rollout_steps(0, min(a.steps, tr.T))
    else:
        tr.fused_rollout = False
        for i in range(a.steps):
            tr.rollout_step(i % tr.T)
    torch.cuda.synchronize()
    tabs = []
    for fn in ("rt_trace_read_policy", "rt_trace_read_env"):
        buf = np.zeros(CAP * SLOTS, np.uint64)
        getattr(L, fn).argtypes = [ctypes.c_void_p]
        assert getattr(L, fn)(buf.ctypes.data) == 0
        tabs.append(buf.reshape(CAP, SLOTS)[:a.envs])
    t = tabs[1].copy()
    if a.two_call:  # the policy stamps live in policy.hip's table
        t[:, 0:2] = tabs[0][:, 0:2]
        t[:, 9] = tabs[0][:, 9]
    t = t.astype(np.int64)
    t0 = t[:, 13].min() if a.persistent else t[:, 0].min()
    us = (t - t0) * 0.01  # 100 MHz
    out = {"mode": a.mode, "envs": a.envs, "phases_us": {}, "kernel_span_us": {}}
    if a.dump:
        np.save(a.dump, us)
    stepped = t[:, 8] > t[:, 5]
    for name, (s0, s1) in PHASES.items():
        d = (us[:, s1] - us[:, s0])[stepped]
        out["phases_us"][name] = {"median": float(np.median(d)), "p90": float(np.percentile(d, 90)),
                                  "max": float(d.max())}
    groups = [np.arange(a.envs) < a.envs // 2, np.arange(a.envs) >= a.envs // 2] if a.pipelined else [None]
    for gi, gm in enumerate(groups):
        sel = np.ones(a.envs, bool) if gm is None else gm
        for k, (s0, s1) in {"k_policy_sample": (0, 1), "k_beam": (2, 4), "k_finish": (5, 8)}.items():
            name = k if gm is None else f"{k}[group {gi}]"
            out["kernel_span_us"][name] = {"first_start": float(us[sel, s0].min()),
                                           "last_start": float(us[sel, s0].max()),
                                           "first_end": float(us[stepped & sel, s1].min()),
                                           "last_end": float(us[sel, s1].max())}
    if a.persistent:  # slots 13/14: each wave's kernel entry / exit
        blk = np.arange(a.envs) // 16
        ent, ext = us[:, 13], us[:, 14]
        out["persistent"] = {"entry_us_pct": [float(np.percentile(ent, q)) for q in (0, 25, 50, 75, 100)],
                             "exit_us_pct": [float(np.percentile(ext, q)) for q in (0, 25, 50, 75, 100)],
                             "life_us_pct": [float(np.percentile(ext - ent, q)) for q in (0, 25, 50, 75, 100)],
                             "blocks_entered_by_us": {str(x): int(np.unique(blk[ent <= x]).size)
                                                      for x in (5, 20, 100, 500, 1000, 2000, 3000)}}
    print(json.dumps(out, indent=1))
    tr.env.close()


if __name__ == "__main__":
    main()
