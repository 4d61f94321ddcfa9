#!/bin/bash
# r03 session 11: sparse wgrad residues for the 16-channel stages; conv1 forward 4-wave blocks A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s11
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RT_C3D_FWD_NTH=256 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py -k "forward or extractor" > $O/pytest_256.log 2>&1 || { tail -60 $O/pytest_256.log; exit 1; }
tail -1 $O/pytest_256.log
for rep in 1 2; do for nth in 512 256; do
  RT_C3D_FWD_NTH=$nth timeout -k 10 300 python -u bench.py --no-cpu --no-update --no-steady --steps 4 --warmup 1 > $O/c3d.json 2>$O/c3d.err || { tail $O/c3d.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/c3d.json').read().strip().splitlines()[-1]); c=d['c3d_mfma']
print('FWD_NTH=$nth train_pass', round(c['train_pass']['ms'],3), 'fwd', round(c['forward']['ms'],3), {k: (round(v['forward_ms'],3), round(v['train_forward_ms'],3), round(v['wgrad_ms'],3)) for k,v in c['stages'].items()})"
done; done
echo ALLDONE
