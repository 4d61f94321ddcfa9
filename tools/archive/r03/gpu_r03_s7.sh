#!/bin/bash
# r03 session 7: sparse weight gradient block shape A/B (512 vs 256 threads, 2- vs 1-row bands)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s7
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "512 2" "256 2" "256 1" "512 2" "256 2" "256 1"; do
  set -- $cfg
  RT_WGS_NT=$1 RT_WGS_PYB=$2 timeout -k 10 300 python -u bench.py --no-cpu --no-update --no-steady --steps 4 --warmup 1 > $O/c3d.json 2>$O/c3d.err || { tail $O/c3d.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/c3d.json').read().strip().splitlines()[-1]); c=d['c3d_mfma']
print('NT=$1 PYB=$2 train_pass', round(c['train_pass']['ms'],3), 'ms', {k: round(v['wgrad_ms'],3) for k,v in c['stages'].items()})"
done
echo ALLDONE
