"""Per-layer forward/backward timings of the C3D encoder (MIOpen, f32)."""
import os
import sys
import time

import torch
import torch.nn as nn

dev = torch.device("cuda")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16


def t(f, n=2):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1000


layers = [("conv1 4->16", nn.Conv3d(4, 16, 3), (B, 4, 64, 64, 64), False),
          ("conv2 16->16 g2", nn.Conv3d(16, 16, 3, groups=2), (B, 16, 31, 31, 31), True),
          ("conv3 16->16 g4", nn.Conv3d(16, 16, 3, groups=4), (B, 16, 14, 14, 14), True),
          ("pool1", nn.MaxPool3d(2, 2), (B, 16, 62, 62, 62), True)]
for name, m, shape, need_dx in layers:
    m = m.to(dev)
    x = torch.rand(shape, device=dev, requires_grad=need_dx)
    fw = t(lambda: m(x))
    y = m(x)
    g = torch.ones_like(y)
    t0 = time.perf_counter()
    torch.autograd.grad(y, [x] + list(m.parameters()) if need_dx else list(m.parameters()) or [x], g,
                        retain_graph=True)
    torch.cuda.synchronize()
    first = time.perf_counter() - t0
    bw = t(lambda: torch.autograd.grad(y, ([x] if need_dx else []) + list(m.parameters()), g, retain_graph=True)
           if (need_dx or list(m.parameters())) else None)
    print(f"B={B} {name:18s} fwd {fw:8.2f} ms  bwd {bw:9.2f} ms  (first bwd {first:.1f}s)", flush=True)
