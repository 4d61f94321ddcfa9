"""conv1/conv2 of the C3D encoder under MIOpen search modes and layouts
(f32): benchmark=False/True, contiguous vs channels_last_3d."""
import sys
import time

import torch
import torch.nn as nn

dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16


def t(f, n=3):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1000


for bench in (False, True):
    torch.backends.cudnn.benchmark = bench
    for cl in (False, True):
        for name, m, shape, need_dx in [("conv1", nn.Conv3d(4, 16, 3), (B, 4, 64, 64, 64), False),
                                        ("conv2", nn.Conv3d(16, 16, 3, groups=2), (B, 16, 31, 31, 31), True)]:
            m = m.to(dev)
            x = torch.rand(shape, device=dev, requires_grad=need_dx)
            if cl:
                m = m.to(memory_format=torch.channels_last_3d)
                x = x.detach().to(memory_format=torch.channels_last_3d).requires_grad_(need_dx)
            fw = t(lambda: m(x))
            y = m(x)
            g = torch.ones_like(y)
            ins = ([x] if need_dx else []) + list(m.parameters())
            bw = t(lambda: torch.autograd.grad(y, ins, g, retain_graph=True))
            print(f"B={B} benchmark={bench} channels_last={cl} {name}: fwd {fw:8.2f} ms bwd {bw:9.2f} ms", flush=True)
