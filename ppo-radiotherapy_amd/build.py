"""Builds librtenv.so (HIP, gfx950) in-tree with hipcc.

The library is the product's compute path; there is no CPU fallback.  It is
built here (cross-compiled, no GPU needed) and travels with the repo to the
GPU box."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "rtenv.hip")
SRCS = [SRC, os.path.join(PKG, "csrc", "policy.hip"), os.path.join(PKG, "csrc", "ppo_update.hip"),
        os.path.join(PKG, "csrc", "c3d.hip")]
HDR = os.path.join(REPO, "include", "rtenv.h")
OUT = os.path.join(PKG, "librtenv.so")
ARCH = os.environ.get("RT_OFFLOAD_ARCH", "gfx950")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
    # every f32/f64 operation must round where the reference rounds
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall", "-Wno-unused-function",
]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build librtenv.so)")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = (*SRCS, HDR, os.path.join(PKG, "csrc", "rt_ddmath.h"), os.path.join(PKG, "csrc", "rt_trace.h"), __file__)
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [hipcc(), *HIPCC_FLAGS, "-I", os.path.join(REPO, "include"), *SRCS, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
