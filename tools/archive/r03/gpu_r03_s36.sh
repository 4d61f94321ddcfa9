#!/bin/bash
# r03 session 36: device hand-off with fewer dose-stream blocks per CU (more slots for the chains) x groups
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s36
mkdir -p $O
for cfg in "0 2 6" "1 2 2" "1 3 2" "1 4 2" "1 2 3" "1 3 3" "1 2 1" "0 2 6"; do
  set -- $cfg
  RT_DENSE_PERSIST=$3 timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --no-update --dense-handoff $1 --rollout-groups $2 > $O/b_h$1_g$2_b$3.json 2> $O/b_h$1_g$2_b$3.err || { tail -20 $O/b_h$1_g$2_b$3.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_h$1_g$2_b$3.json')); r=d['roofline']; print('handoff $1 groups $2 bpc $3', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['frac'],3))"
done
echo ALLDONE
