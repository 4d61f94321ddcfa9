#!/bin/bash
# round 6: the pipelined rollout with the finish of step t-1 fused into step
# t's policy launch (k_step_policy<false, true>): bitwise gates, then the
# driver's bench command (rollout only) twice
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_prefin; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_trainer.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  python3 - $O/b$i.json $i <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
s = d["steady_state"]; r = d["roofline"]
print("prefin", sys.argv[2], "value %.3f M" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "steady %.4f" % s["ms_per_step"],
      "kms", {k: round(v, 4) for k, v in r["kernel_ms_all"].items()}, "frac", round(r["frac"], 3))
PY
done
echo ALLDONE
