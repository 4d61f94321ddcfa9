#!/bin/bash
# round 6: k_dense blocks per CU x policy envs per block in the pipelined
# rollout (experiment knobs RT_X_PIPE_BPC / RT_X_PIPE_WPB): room for one chain
# wave per SIMD beside 4 stream waves
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_bpcwpb; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/b$n.json 2> $O/b$n.err || { tail -20 $O/b$n.err; exit 1; }
  python3 - $O/b$n.json $n <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
s = d["steady_state"]; r = d["roofline"]
print(sys.argv[2], "value %.3f M" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "steady %.4f" % s["ms_per_step"],
      "kms", {k: round(v, 4) for k, v in r["kernel_ms_all"].items()})
PY
}
for cfg in ${CFGS:-5:8 4:4 4:2 5:4 4:8 3:4 5:8}; do
  b=${cfg%:*}; w=${cfg#*:}
  run bpc${b}_wpb${w} RT_X_PIPE_BPC=$b RT_X_PIPE_WPB=$w
done
echo ALLDONE
