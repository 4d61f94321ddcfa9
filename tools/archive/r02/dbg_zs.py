"""Debug: conv2 forward outputs (values, argmax bytes) on the backward test's
data at 63^3, saved for an A/B comparison between RT_C3D_ZS builds."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402

from ppo_radiotherapy_amd import _lib  # noqa: E402

dims, groups, cin, B = (63, 63, 63), 2, 16, 2
g = torch.Generator().manual_seed(7 + cin + groups)
x = torch.rand((B, cin, *dims), generator=g)
x = torch.relu(x - 0.3)
w = torch.randn((16, cin // groups, 3, 3, 3), generator=g) * (1.0 / np.sqrt(cin // groups * 27))
b = torch.randn(16, generator=g) * 0.1
L = _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(0, 0, 0))
lib = _lib.load()
od = (ctypes.c_int32 * 3)()
_lib.check(lib.rt_conv_out_dims(ctypes.byref(L), od), "dims")
dev = torch.device("cuda")
xd, wd, bd = x.to(dev), w.to(dev), b.to(dev)
y = torch.full((B, 16, *od), float("nan"), device=dev)
am = torch.full((B, 16, *od), 255, dtype=torch.uint8, device=dev)
_lib.check(lib.rt_conv_relu_pool_fwd(ctypes.byref(L), B, xd.data_ptr(), None, wd.data_ptr(), bd.data_ptr(),
                                     y.data_ptr(), am.data_ptr(), None), "fwd")
torch.cuda.synchronize()
os.makedirs("gpurun_out/dbg", exist_ok=True)
tag = os.environ.get("RT_C3D_ZS", "1")
np.save(f"gpurun_out/dbg/y_{tag}.npy", y.cpu().numpy())
np.save(f"gpurun_out/dbg/am_{tag}.npy", am.cpu().numpy())
print(tag, "nan", int(torch.isnan(y).sum()), "unwritten am", int((am == 255).sum()))
