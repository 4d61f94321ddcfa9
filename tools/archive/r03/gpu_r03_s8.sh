#!/bin/bash
# r03 session 8: sparse weight gradient loop variants (1 vs 2 windows per iteration) x block shape
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RT_LIB_PATH=$PWD/_variants/librtenv_wgsu2.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py -k backward > $O/pytest_u2.log 2>&1 || { tail -60 $O/pytest_u2.log; exit 1; }
tail -1 $O/pytest_u2.log
for rep in 1 2; do
for lib in default wgsu2; do
for nt in 256 512; do
  if [ $lib = default ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/_variants/librtenv_$lib.so; fi
  RT_WGS_NT=$nt timeout -k 10 300 python -u bench.py --no-cpu --no-update --no-steady --steps 4 --warmup 1 > $O/c3d.json 2>$O/c3d.err || { tail $O/c3d.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/c3d.json').read().strip().splitlines()[-1]); c=d['c3d_mfma']
print('$lib NT=$nt train_pass', round(c['train_pass']['ms'],3), 'ms', {k: round(v['wgrad_ms'],3) for k,v in c['stages'].items()})"
done; done; done
unset RT_LIB_PATH
echo ALLDONE
