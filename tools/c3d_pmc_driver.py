"""Runs each C3D stage kernel a few times at 64^3 (batch 64) -- a target for
rocprofv3 --pmc (tools/bench_c3d_kernels.py times them); C3D_PMC_B sets the batch."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402

from ppo_radiotherapy_amd import _lib  # noqa: E402

B = int(os.environ.get("C3D_PMC_B", "64"))
dev = torch.device("cuda")
L = _lib.load()
for cin, groups, dims in [(4, 1, (64, 64, 64)), (16, 2, (31, 31, 31)), (16, 4, (14, 14, 14))]:
    x = torch.rand((B, cin, *dims), device=dev)
    w = torch.randn((16, cin // groups, 3, 3, 3), device=dev) * 0.1
    b = torch.randn(16, device=dev) * 0.1
    lay = _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(0, 0, 0))
    od = (ctypes.c_int32 * 3)()
    L.rt_conv_out_dims(ctypes.byref(lay), od)
    y = torch.empty((B, 16, *od), device=dev)
    am = torch.empty((B, 16, *od), dtype=torch.uint8, device=dev)
    gy = torch.randn_like(y)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    ws = torch.empty(int(L.rt_conv_wgrad_workspace_floats(ctypes.byref(lay), B)), device=dev)
    for _ in range(3):
        L.rt_conv_relu_pool_fwd(ctypes.byref(lay), B, x.data_ptr(), None, w.data_ptr(), b.data_ptr(), y.data_ptr(),
                                am.data_ptr(), None)
        L.rt_conv_relu_pool_wgrad(ctypes.byref(lay), B, x.data_ptr(), None, gy.data_ptr(), am.data_ptr(),
                                  dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(), None)
        if cin == 16:  # the grouped stages also get the data gradient
            dx = torch.empty_like(x)
            L.rt_conv_relu_pool_dgrad(ctypes.byref(lay), B, w.data_ptr(), gy.data_ptr(), am.data_ptr(),
                                      dx.data_ptr(), None)
torch.cuda.synchronize()
print("ok")
