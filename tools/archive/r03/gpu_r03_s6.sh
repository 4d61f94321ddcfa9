#!/bin/bash
# r03 session 6: sparse weight gradient with 8-B pair reads: C3D tests + stage timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s6
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_vision.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu --no-update --no-steady --steps 8 --warmup 2 > $O/c3d.json 2>$O/c3d.err || { tail $O/c3d.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/c3d.json').read().strip().splitlines()[-1]); c=d['c3d_mfma']
print('train_pass', round(c['train_pass']['ms'],3), 'ms', round(c['train_pass']['achieved'],1), 'TF/s', {k: round(v['wgrad_ms'],3) for k,v in c['stages'].items()})"
echo ALLDONE
