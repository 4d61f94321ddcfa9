#!/bin/bash
# round 6: CU-split pipelined rollout, one chain stream; sweep of the split and
# of a chain stream allowed on every CU (RT_PIPE_CHAIN_ALL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_split2; mkdir -p $O
RT_PIPE_CHAIN_CUS=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest64.log 2>&1 || { tail -30 $O/pytest64.log; exit 1; }
tail -2 $O/pytest64.log
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
run base RT_PIPE_CHAIN_CUS=0
run c64 RT_PIPE_CHAIN_CUS=64
run c64all RT_PIPE_CHAIN_CUS=64 RT_PIPE_CHAIN_ALL=1
run c32all RT_PIPE_CHAIN_CUS=32 RT_PIPE_CHAIN_ALL=1
run c128 RT_PIPE_CHAIN_CUS=128
run base2 RT_PIPE_CHAIN_CUS=0
echo ALLDONE
