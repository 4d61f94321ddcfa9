#!/bin/bash
# r03 session 4: the sparse (argmax-gather) C3D weight gradient: stage / extractor /
# vision tests, then the C3D stage timing A/B (dense MFMA ring vs sparse)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s4
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_configs.py tests/test_gpu_vision.py tests/test_gpu_dp.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for v in 0 1; do
  RT_C3D_WGSPARSE=$v timeout -k 10 300 python -u bench.py --no-cpu --no-update --no-steady --steps 8 --warmup 2 > $O/c3d_$v.json 2>$O/c3d.err || { tail $O/c3d.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/c3d_$v.json').read().strip().splitlines()[-1]); c=d['c3d_mfma']
print('WGSPARSE=$v train_pass', round(c['train_pass']['ms'],3), 'ms', round(c['train_pass']['achieved'],1), 'TF/s', {k: round(v['wgrad_ms'],3) for k,v in c['stages'].items()})"
done
RT_C3D_WGSPARSE=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu --no-update --no-steady --steps 8 --warmup 2 > $O/kt.json 2>$O/kt.err || { tail $O/kt.err; exit 1; }
grep -E "wgrad|conv" $O/kt/run_kernel_stats.csv | cut -c1-200
find $O -name "*.db" -delete
echo ALLDONE
