#!/bin/bash
# r05 session 2: persistent dense rollout (rollout groups 0) with a cohort
# phase stagger -- bitwise gate (test_gpu_rollout) on the in-tree build, then
# a sweep of variant builds (cohorts x delay x loads in flight) against the
# two-group pipeline, bench windows only (no update / C3D / CPU legs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest_rollout.log 2>&1 || { tail -40 $O/pytest_rollout.log; exit 1; }
tail -1 $O/pytest_rollout.log
B="--no-cpu --no-c3d --no-update --steps 20 --warmup 4"
timeout -k 10 300 python3 bench.py $B --rollout-groups 2 > $O/g2.json 2> $O/g2.err || { tail -20 $O/g2.err; exit 1; }
for v in c1 c2d60 c4d30 c4d50 c4d70 c4d30u8; do
  RT_LIB_PATH=_variants/librtenv_$v.so timeout -k 10 300 python3 bench.py $B --rollout-groups 0 > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
done
timeout -k 10 300 python3 bench.py $B --rollout-groups 0 > $O/intree_g0.json 2> $O/intree_g0.err || { tail -20 $O/intree_g0.err; exit 1; }
python3 - <<'PY'
import json
O = "gpurun_out/r05_s2"
for v in ["g2", "c1", "c2d60", "c4d30", "c4d50", "c4d70", "c4d30u8", "intree_g0"]:
    d = json.load(open(f"{O}/{v}.json")); s = d["steady_state"]
    print(f"{v:10s} value {d['value']/1e6:7.3f} M  {d['ms_per_step']:.4f} ms  steady {s['env_steps_per_s']/1e6:7.3f} M {s['ms_per_step']:.4f} ms  windows {[round(x/1e6,2) for x in s['windows_env_steps_per_s']]}")
PY
echo ALLDONE
