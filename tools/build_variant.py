"""Build a kernel-variant librtenv.so for A/B runs (RT_LIB_PATH selects it):
one source recompiled with extra flags, the other objects from the in-tree
build.

    python tools/build_variant.py NAME c3d.hip -DRT_C3D_EXP=1 [...]
    -> _variants/librtenv_NAME.so
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: E402,F401
from ppo_radiotherapy_amd import build as B  # noqa: E402


def main():
    name, src_base, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build()
    src = [s for s in B.SRCS if os.path.basename(s) == src_base][0]
    vdir = os.path.join(B.REPO, "_variants")
    os.makedirs(vdir, exist_ok=True)
    obj = os.path.join(vdir, f"{name}_{os.path.splitext(src_base)[0]}.o")
    subprocess.run([B.hipcc(), *B.HIPCC_FLAGS, *B.EXTRA_FLAGS.get(src, []), *extra, "-I",
                    os.path.join(B.REPO, "include"), "-c", src, "-o", obj], check=True)
    objs = [obj if s == src else os.path.join(B.OBJ_DIR, os.path.splitext(os.path.basename(s))[0] + ".o")
            for s in B.SRCS]
    out = os.path.join(vdir, f"librtenv_{name}.so")
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", out], check=True)
    print(out)


if __name__ == "__main__":
    main()
