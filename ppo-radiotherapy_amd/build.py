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
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
    # every f32/f64 operation must round where the reference rounds
    "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
    "-Wall", "-Wno-unused-function",
]
# per-source extra flags.  rtenv.hip: machine LICM hoists the f64 series
# constants of the pose update out of k_rollout_policy's step loop and spills
# them to scratch (reloaded serially inside the sincos chain); without it the
# kernel fits 128 VGPRs with no spill, and the other kernels' loops are unchanged
# (register renaming only).  c3d.hip: no SLP vectorizer -- it packs f32 adds
# and FMAs into v_pk_add_f32 / v_pk_fma_f32, which beside MFMAs cost more issue
# than the scalar pairs (MI355X_MICROARCH.md); without it the conv1 sparse
# weight gradient runs 3.5 % and the groups-2 data gradient 2 % faster
# (profiles/r05/r05_s19_c3d_slp.txt).
EXTRA_FLAGS = {SRC: ["-mllvm", "-disable-machine-licm"], SRCS[3]: ["-fno-slp-vectorize"]}
OBJ_DIR = os.path.join(PKG, "_obj")


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build librtenv.so)")


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = (*SRCS, HDR, *(os.path.join(PKG, "csrc", h) for h in ("rt_ddmath.h", "rt_trace.h", "policy_core.h")),
            __file__)
    return any(os.path.getmtime(p) > t for p in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not needs_build():
        return OUT
    os.makedirs(OBJ_DIR, exist_ok=True)
    procs, objs = [], []
    for src in SRCS:
        obj = os.path.join(OBJ_DIR, os.path.splitext(os.path.basename(src))[0] + ".o")
        cmd = [hipcc(), *HIPCC_FLAGS, *EXTRA_FLAGS.get(src, []), "-I", os.path.join(REPO, "include"), "-c", src,
               "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((subprocess.Popen(cmd), cmd))
        objs.append(obj)
    for p, cmd in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
