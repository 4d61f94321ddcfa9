"""C3D (FeaturesExtractor3D) timings on MI355X, printing as it goes."""
import os
import sys
import time

import torch

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
import _rtpkg  # noqa
from ppo_radiotherapy_amd.networks import FeaturesExtractor3D  # noqa


def t(f, n=3):
    f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1000


dev = torch.device("cuda")
for B in [int(x) for x in (sys.argv[1:] or ["8", "64"])]:
    fe = FeaturesExtractor3D((4, 64, 64, 64), 64).to(dev)
    x = torch.rand(B, 4, 64, 64, 64, device=dev)
    t0 = time.perf_counter()
    with torch.no_grad():
        fe(x)
    torch.cuda.synchronize()
    print(f"B={B} first fwd (incl. MIOpen setup) {time.perf_counter() - t0:.1f}s", flush=True)
    with torch.no_grad():
        ms = t(lambda: fe(x))
    gf = 0.999 * B
    print(f"B={B} fwd {ms:.2f} ms  {gf / ms:.1f} TFLOP/s", flush=True)
    conv1 = fe.cnn[0]
    with torch.no_grad():
        ms1 = t(lambda: conv1(x))
    print(f"B={B} conv1 fwd {ms1:.2f} ms  {2 * B * 16 * 62**3 * 4 * 27 / ms1 / 1e9:.1f} TFLOP/s", flush=True)
    x.requires_grad_(False)
    t0 = time.perf_counter()
    fe(x).sum().backward()
    torch.cuda.synchronize()
    print(f"B={B} first fwd+bwd {time.perf_counter() - t0:.1f}s", flush=True)
    ms = t(lambda: fe(x).sum().backward(), n=2)
    print(f"B={B} fwd+bwd {ms:.2f} ms", flush=True)
