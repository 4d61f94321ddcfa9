"""Build a kernel-variant librtenv.so for A/B runs (RT_LIB_PATH selects it):
one source recompiled with extra flags, the other objects from the in-tree
build.

    python tools/build_variant.py NAME rtenv.hip -DRT_PIPE_DENSE_BPC=4 [...]
    -> _variants/librtenv_NAME.so
    python tools/build_variant.py NAME c3d.hip --rev HEAD [...]
    (the source as of a git revision: before/after A/B of an edit)
    python tools/build_variant.py NAME c3d.hip --file /tmp/c3d_alt.hip [...]
    (another text of the source, compiled beside it)
"""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: E402,F401
from ppo_radiotherapy_amd import build as B  # noqa: E402


def main():
    name, src_base, extra = sys.argv[1], sys.argv[2], sys.argv[3:]
    rev = alt = None
    if "--file" in extra:
        i = extra.index("--file")
        alt = extra[i + 1]
        del extra[i:i + 2]
    if "--rev" in extra:
        i = extra.index("--rev")
        rev = extra[i + 1]
        del extra[i:i + 2]
    B.build()
    src = [s for s in B.SRCS if os.path.basename(s) == src_base][0]
    vdir = os.path.join(B.REPO, "_variants")
    os.makedirs(vdir, exist_ok=True)
    csrc = src
    if rev or alt:  # compile the other text next to the source (same include paths)
        csrc = os.path.join(os.path.dirname(src), f"_rev_{name}_{src_base}")
        if alt:
            with open(alt) as f:
                text = f.read()
        else:
            text = subprocess.run(["git", "-C", B.REPO, "show", f"{rev}:{os.path.relpath(src, B.REPO)}"],
                                  check=True, capture_output=True, text=True).stdout
        with open(csrc, "w") as f:
            f.write(text)
    obj = os.path.join(vdir, f"{name}_{os.path.splitext(src_base)[0]}.o")
    try:
        subprocess.run([B.hipcc(), *B.HIPCC_FLAGS, *B.EXTRA_FLAGS.get(src, []), *extra, "-I",
                        os.path.join(B.REPO, "include"), "-c", csrc, "-o", obj], check=True)
    finally:
        if rev or alt:
            os.remove(csrc)
    objs = [obj if s == src else os.path.join(B.OBJ_DIR, os.path.splitext(os.path.basename(s))[0] + ".o")
            for s in B.SRCS]
    out = os.path.join(vdir, f"librtenv_{name}.so")
    subprocess.run([B.hipcc(), f"--offload-arch={B.ARCH}", "-shared", "-fPIC", *objs, "-o", out], check=True)
    print(out)


if __name__ == "__main__":
    main()
