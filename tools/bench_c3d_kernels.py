"""C3D stage kernels (csrc/c3d.hip) vs MIOpen (torch conv3d + relu + max_pool3d),
f32, 64^3 vision shapes: time per call and TFLOP/s (conv FLOPs, dense)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from ppo_radiotherapy_amd import _lib  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda")
L = _lib.load()
S = 64


def tm(f, n=5):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


out = {}
for name, cin, groups, dims in [("conv1", 4, 1, (S, S, S)), ("conv2", 16, 2, (31, 31, 31)),
                                ("conv3", 16, 4, (14, 14, 14))]:
    x = torch.rand((B, cin, *dims), device=dev)
    w = torch.randn((16, cin // groups, 3, 3, 3), device=dev) * 0.1
    b = torch.randn(16, device=dev) * 0.1
    lay = _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(0, 0, 0))
    od = (ctypes.c_int32 * 3)()
    L.rt_conv_out_dims(ctypes.byref(lay), od)
    y = torch.empty((B, 16, *od), device=dev)
    am = torch.empty((B, 16, *od), dtype=torch.uint8, device=dev)
    st = _lib.stream_handle()
    ours = tm(lambda: _lib.check(L.rt_conv_relu_pool_fwd(ctypes.byref(lay), B, x.data_ptr(), None, w.data_ptr(),
                                                         b.data_ptr(), y.data_ptr(), am.data_ptr(), st), "fwd"))
    miop = tm(lambda: F.max_pool3d(F.relu(F.conv3d(x, w, b, groups=groups)), 2, 2))
    flops = 2 * B * 16 * (cin // groups) * 27 * (dims[0] - 2) * (dims[1] - 2) * (dims[2] - 2)
    out[name] = {"ours_ms": ours * 1e3, "miopen_ms": miop * 1e3, "ours_tflops": flops / ours / 1e12,
                 "miopen_tflops": flops / miop / 1e12}
    gy = torch.randn_like(y)
    dw = torch.empty_like(w)
    db = torch.empty_like(b)
    ws = torch.empty(int(L.rt_conv_wgrad_workspace_floats(ctypes.byref(lay), B)), device=dev)
    wg = tm(lambda: _lib.check(L.rt_conv_relu_pool_wgrad(ctypes.byref(lay), B, x.data_ptr(), None, gy.data_ptr(),
                                                         am.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(),
                                                         ws.numel(), st), "wgrad"))
    out[name]["wgrad_ms"] = wg * 1e3
    out[name]["wgrad_tflops"] = flops / wg / 1e12
    if cin == 16:
        dx = torch.empty_like(x)
        dg = tm(lambda: _lib.check(L.rt_conv_relu_pool_dgrad(ctypes.byref(lay), B, w.data_ptr(), gy.data_ptr(),
                                                             am.data_ptr(), dx.data_ptr(), st), "dgrad"))
        out[name]["dgrad_ms"] = dg * 1e3
        out[name]["dgrad_tflops"] = flops / dg / 1e12

# the whole extractor, forward + backward (a training micro-batch), and inference forward
from ppo_radiotherapy_amd.networks import FeaturesExtractor3D  # noqa: E402

fe = FeaturesExtractor3D((4, S, S, S), 64).to(dev)
xo = torch.rand((B, 4, S, S, S), device=dev)


def train_step():
    fe.zero_grad(set_to_none=True)
    fe(xo).sum().backward()


out["extractor_fwd_bwd_ms"] = tm(train_step) * 1e3
with torch.no_grad():
    out["extractor_fwd_ms"] = tm(lambda: fe(xo)) * 1e3
out["gflop_per_sample_fwd"] = 2 * (16 * 4 * 27 * (S - 2) ** 3 + 16 * 8 * 27 * 29 ** 3 + 16 * 4 * 27 * 12 ** 3) / 1e9
print(json.dumps({"batch": B, **out}))
