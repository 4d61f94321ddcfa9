"""Grouped C3D stage forwards (conv2 groups=2 on 31^3, conv3 groups=4 on
14^3 -- the 64^3 vision shapes; --big: the 128^3 shapes 63^3 / 30^3) at batch
B: ms per call, inference and training (argmax) variants and the data gradient.  RT_C3D_ZS=0
selects the dense ring kernel (A/B)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402

from ppo_radiotherapy_amd import _lib  # noqa: E402


def main():
    B = 512
    big = "--big" in sys.argv
    dev = torch.device("cuda")
    L = _lib.load()
    out = {}
    for name, groups, S in (("conv2", 2, 63 if big else 31), ("conv3", 4, 30 if big else 14)):
        layer = _lib.RtConvLayer(16, groups, (ctypes.c_int32 * 3)(S, S, S), (ctypes.c_int32 * 3)(0, 0, 0))
        od = (ctypes.c_int32 * 3)()
        _lib.check(L.rt_conv_out_dims(ctypes.byref(layer), od), "dims")
        x = torch.rand(B, 16, S, S, S, device=dev)
        w = torch.randn(16, 16 // groups, 3, 3, 3, device=dev) * 0.1
        b = torch.randn(16, device=dev) * 0.1
        y = torch.empty(B, 16, *od, device=dev)
        am = torch.empty(B, 16, *od, dtype=torch.uint8, device=dev)
        res = {}
        gy = torch.randn_like(y)
        dx = torch.empty_like(x)
        _lib.check(L.rt_conv_relu_pool_fwd(ctypes.byref(layer), B, x.data_ptr(), None, w.data_ptr(), b.data_ptr(),
                                           y.data_ptr(), am.data_ptr(), None), "fwd")

        def fd():
            _lib.check(L.rt_conv_relu_pool_dgrad(ctypes.byref(layer), B, w.data_ptr(), gy.data_ptr(), am.data_ptr(),
                                                 dx.data_ptr(), None), "dgrad")
        fd()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fd()
        torch.cuda.synchronize()
        res["dgrad"] = 1e3 * (time.perf_counter() - t0) / 10
        for train in (False, True):
            def f():
                _lib.check(L.rt_conv_relu_pool_fwd(ctypes.byref(layer), B, x.data_ptr(), None, w.data_ptr(),
                                                   b.data_ptr(), y.data_ptr(), am.data_ptr() if train else None,
                                                   None), "fwd")
            f()
            torch.cuda.synchronize()
            n = 10
            t0 = time.perf_counter()
            for _ in range(n):
                f()
            torch.cuda.synchronize()
            res["train" if train else "infer"] = 1e3 * (time.perf_counter() - t0) / n
        out[name] = res
    print(json.dumps({"zs": os.environ.get("RT_C3D_ZS", "1"), "big": big, **out}))


if __name__ == "__main__":
    main()
