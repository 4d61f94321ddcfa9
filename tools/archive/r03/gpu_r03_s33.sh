#!/bin/bash
# r03 session 33: A/B of the latency chain's wave priority (RT_CHAIN_PRIO=3 build) on the default rollout
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s33
mkdir -p $O
for v in base prio3 base prio3; do
  if [ $v = base ]; then L=""; else L="$PWD/_variants/librtenv_$v.so"; fi
  RT_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --no-update > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms')"
done
echo ALLDONE
