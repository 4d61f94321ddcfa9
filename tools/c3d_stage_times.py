"""bench.py's c3d_mfma object alone (configs[3]'s C3D stage kernels on 512
vision observations at 64^3, f32 and bf16x3 forward products), printed as a
compact per-stage table plus the JSON object.  Usage: python tools/c3d_stage_times.py [grid]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO]
import _rtpkg  # noqa: E402,F401
import torch  # noqa: E402

import bench  # noqa: E402
from ppo_radiotherapy_amd import assets  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
lib = assets.synthetic_library((S, S, S), 1000, 0)
r = bench.c3d_roofline(dev, lib, (S, S, S))
for prec, st in (("f32", r["stages"]), ("bf16x3", r["bf16x3"]["stages"])):
    for k, v in st.items():
        print(f"{prec:7s} {k}: fwd {v['forward_ms']:.3f} ms"
              + (f" ({v['forward_frac']:.3f} of f32 peak executed)" if "forward_frac" in v else "")
              + f" | train fwd {v['train_forward_ms']:.3f} | wgrad {v['wgrad_ms']:.3f}"
              + (f" (VALU {v['wgrad_valu_frac']:.3f})" if "wgrad_valu_frac" in v else "")
              + (f" | dgrad {v['dgrad_ms']:.3f}" if "dgrad_ms" in v else "")
              + (f" ({v['dgrad_frac']:.3f})" if "dgrad_frac" in v else ""))
print(f"f32 forward {r['forward']['ms']:.3f} ms = {r['forward']['achieved']:.1f} TF executed ({r['forward']['frac']:.3f}); "
      f"train pass {r['train_pass']['ms']:.3f} ms ({r['train_pass']['frac']:.3f} executed); "
      f"bf16x3 train pass {r['bf16x3']['train_pass_ms']:.3f} ms")
print(json.dumps(r))
