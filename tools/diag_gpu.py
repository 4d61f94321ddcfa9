"""GPU-box diagnostics: loaded HIP runtimes, device count, pose parity stats."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _rtpkg  # noqa
from ppo_radiotherapy_amd import _lib

print("torch", torch.__version__, "cuda avail", torch.cuda.is_available(), torch.cuda.device_count())
L = _lib.load()
maps = open("/proc/self/maps").read().splitlines()
libs = sorted({l.split()[-1] for l in maps if ("amdhip" in l or "hsa-runtime" in l)})
print("loaded:", libs)
h = ctypes.CDLL("libamdhip64.so.7")
n = ctypes.c_int(-1)
rc = h.hipGetDeviceCount(ctypes.byref(n))
print("hipGetDeviceCount rc", rc, "n", n.value)
z = np.load(os.path.join(REPO, "tests/golden/transform_cases.npz"))
m = len(z["rot_action"])
dev = torch.device("cuda", 0)
pos = np.tile(np.array([33.5, 21.5, 35.0]), (m, 1))
act = np.zeros((m, 6), np.float32)
act[:, 3:] = z["rot_action"]
p = torch.tensor(pos, dtype=torch.float64, device=dev)
d = torch.tensor(z["rot_dir_in"], dtype=torch.float64, device=dev)
a = torch.tensor(act, device=dev)
out = torch.zeros((m, 10), dtype=torch.float64, device=dev)
_lib.check(L.rt_debug_pose(_lib.grid_arg((67, 43, 70)), m, p.data_ptr(), d.data_ptr(), a.data_ptr(), out.data_ptr(), None), "pose")
o = out.cpu().numpy()
bad = np.any(o[:, 3:6] != z["rot_dir_out"], axis=1)
print("rot dir mismatches", bad.sum(), "of", m, "max abs diff", np.abs(o[:, 3:6] - z["rot_dir_out"]).max())
ulps = np.abs(o[:, 3:6].view(np.int64) - z["rot_dir_out"].view(np.int64)).max()
print("max ulp diff", ulps)
small = np.abs(z["rot_action"]).max(axis=1) < 1e-3
print("mismatch among small-angle cases", bad[small].sum(), "/", small.sum())
# device sin/cos vs host
x = np.random.default_rng(0).uniform(0, 3, 200000)
print("(host libm comparison of sin/cos would need a kernel)")
