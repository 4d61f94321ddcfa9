#!/bin/bash
# r05 session 6: the dataflow rollout (RT_ROLLOUT_FLOW = 16) -- bitwise vs the
# stepwise launches, then bench windows vs the two-group pipeline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py -k "16 or rejects" > $O/pytest_flow.log 2>&1
rc=$?; tail -15 $O/pytest_flow.log; [ $rc -eq 0 ] || exit 1
B="--no-cpu --no-c3d --no-update --steps 20 --warmup 4"
timeout -k 10 300 python3 bench.py $B --rollout-groups 16 > $O/g16.json 2> $O/g16.err || { tail -20 $O/g16.err; exit 1; }
timeout -k 10 300 python3 bench.py $B --rollout-groups 2 > $O/g2.json 2> $O/g2.err || { tail -20 $O/g2.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_s6"
for v in ["g16", "g2"]:
    d = json.load(open(f"{O}/{v}.json")); s = d["steady_state"]
    print(f"{v:5s} value {d['value']/1e6:7.3f} M  {d['ms_per_step']:.4f} ms  steady {s['env_steps_per_s']/1e6:7.3f} M {s['ms_per_step']:.4f} ms  timed {d['roofline']['timed_pass_ms_per_step']:.4f}")
PY
echo ALLDONE
