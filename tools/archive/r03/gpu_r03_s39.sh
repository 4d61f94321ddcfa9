#!/bin/bash
# r03 session 39: default bench with the rocprof cross-check field
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s39
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M frac', round(r['frac'],3), 'rocprof', r.get('rocprof')); print('c3d bf16x3 fwd', round(d['c3d_mfma']['bf16x3']['forward_ms'],3)); print('cpu', d['cpu_baseline']['value'])"
echo ALLDONE
