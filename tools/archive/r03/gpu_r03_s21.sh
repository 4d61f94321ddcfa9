#!/bin/bash
# r03 session 21: device hand-off of the pipelined dense rollout (k_dense_rollout):
# bitwise rollout tests, then bench A/B of events vs device hand-off over 2/3/4 groups
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s21
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for cfg in "0 2" "1 2" "1 3" "1 4" "0 2" "1 3"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --no-update --dense-handoff $1 --rollout-groups $2 > $O/b_h$1_g$2.json 2> $O/b_h$1_g$2.err || { tail -20 $O/b_h$1_g$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_h$1_g$2.json')); r=d['roofline']; print('handoff $1 groups $2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['frac'],3), round(r['step_frac_of_hbm'],3))"
done
echo ALLDONE
