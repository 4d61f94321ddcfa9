#!/bin/bash
# r03 session 42: k_finish early loads of the tail (RT_FINISH_PF): parity tests, A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s42
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headline.py tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_fused_step.py tests/test_gpu_vision.py tests/test_gpu_configs.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in pf1 pf0 pf1 pf0 pf1 pf0; do
  if [ $v = pf1 ]; then L=""; else L="$PWD/_variants/librtenv_$v.so"; fi
  RT_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --no-update > $O/b_$v.json 2> $O/b_$v.err || { tail -20 $O/b_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$v.json')); print('$v', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', round(d['roofline']['kernel_ms_all']['k_finish'],4))"
done
echo ALLDONE
