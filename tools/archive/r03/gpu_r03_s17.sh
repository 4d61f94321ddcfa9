#!/bin/bash
# r03 session 17: bf16x3 with round-to-nearest hi; error report and update time, 3 vs 4 terms (RT_BF16_TERMS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s17
mkdir -p $O
for lib in default t4; do
  if [ $lib = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/_variants/librtenv_$lib.so; fi
  timeout -k 10 120 python -u tools/prec_report.py $O/prec_$lib.json || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --steps 16 --warmup 4 > $O/u.json 2>$O/u.err || { tail $O/u.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/u.json').read().strip().splitlines()[-1]); print('$lib f32', round(d['ppo_update_ms']*1000,2), 'bf16x3', round(d['ppo_update_ms_bf16x3']*1000,2), 'us/minibatch')"
done
