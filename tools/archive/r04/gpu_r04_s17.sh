#!/bin/bash
# r04 session 17: the incremental persistent rollout with wave issue priority
# rotated per step (parity + A/B vs prev, three runs each, raw stamps)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s17
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_fused_step.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
for v in prev new; do
  if [ $v = prev ]; then export RT_LIB_PATH=_variants/librtenv_prev.so; else unset RT_LIB_PATH; fi
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update --no-steady --step-mode incremental > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; print('$v', $rep, 'incr value', round(d['value']/1e6,2), 'M', round(d['ms_per_step']*1000,1), 'us/step frac', round(r.get('frac',0),3), 'dense', round(d['other_step_mode']['env_steps_per_s']/1e6,2))"
done
done
unset RT_LIB_PATH
timeout -k 10 300 python3 tools/trace_env.py --mode incremental --persistent --steps 24 --dump $O/stamps_incr.npy > $O/trace_incr.json 2> $O/trace_incr.err || { tail -30 $O/trace_incr.err; exit 1; }
python3 - <<'PY'
import json, numpy as np
us = np.load("gpurun_out/r04_s17/stamps_incr.npy")
life = us[:, 14] - us[:, 13]
w = np.arange(us.shape[0]) % 16
print("life pct", np.percentile(life, [0, 50, 90, 100]).round(0), "by age rank", [round(life[(w >> 2) == k].mean()) for k in range(4)])
PY
echo ALLDONE
