#!/bin/bash
# round 6: policy-kernel envs per block in the pipelined dense rollout beside
# the 16-row stream (variant builds: w2 / w4 / w16; the tree: 8), driver bench
# without cpu / c3d / update, alternated
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06_wpb
mkdir -p $O
for i in 1 2; do
  for t in w8 w2 w4 w16; do
    L=""; [ $t != w8 ] && L=$PWD/_var6/librtenv_$t.so
    RT_LIB_PATH=$L timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/${t}_$i.json 2> $O/${t}_$i.err || { tail $O/${t}_$i.err; exit 1; }
  done
done
python3 - $O <<'PY'
import json, sys
O = sys.argv[1]
for t in ("w8", "w2", "w4", "w16"):
    for i in (1, 2):
        d = json.loads([l for l in open(f"{O}/{t}_{i}.json") if l.startswith("{")][-1]); r = d["roofline"]; s = d.get("steady_state", {})
        print(t, i, "value", round(d["value"] / 1e6, 3), "ms", round(d["ms_per_step"], 4), "steady", s.get("ms_per_step"),
              "kms", r.get("kernel_ms_all"))
PY
