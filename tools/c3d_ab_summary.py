"""Summarise tools/archive/gpu_c3d_ab.sh logs: per variant, per stage ms (min over passes)."""
import glob
import json
import os
import sys

d = sys.argv[1]
res = {}
for f in sorted(glob.glob(os.path.join(d, "librtenv_c3d_*_*.log"))):
    v = os.path.basename(f).rsplit("_", 1)[0].replace("librtenv_c3d_", "")
    try:
        j = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:  # noqa: BLE001
        continue
    row = {f"{s}.{k}": j[s][k] for s in ("conv1", "conv2", "conv3") for k in ("ours_ms", "wgrad_ms", "dgrad_ms")
           if k in j.get(s, {})}
    row["ext_fwd"] = j["extractor_fwd_ms"]
    row["ext_fwd_bwd"] = j["extractor_fwd_bwd_ms"]
    r = res.setdefault(v, {})
    for k, x in row.items():
        r[k] = min(r.get(k, 1e9), x)
keys = sorted({k for r in res.values() for k in r})
print("variant".ljust(14) + "".join(k[-14:].rjust(15) for k in keys))
for v, r in res.items():
    print(v.ljust(14) + "".join(f"{r.get(k, float('nan')):15.3f}" for k in keys))
