#!/bin/bash
# round 6: chain kernels and the lung stream on separate library streams, the
# chain at the greatest stream priority (RT_PIPE_PRIO=1) or both default (0),
# against the two-group ring (unset)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_prio; mkdir -p $O
RT_PIPE_PRIO=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {
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
run ring RT_X_NONE=1
run prio1 RT_PIPE_PRIO=1
run prio0 RT_PIPE_PRIO=0
run prio1b RT_PIPE_PRIO=1
run ring2 RT_X_NONE=1
echo ALLDONE
