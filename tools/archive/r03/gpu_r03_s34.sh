#!/bin/bash
# r03 session 34: k_finish tumour gather batched (RT_FINISH_KG): parity tests, A/B with events and device hand-off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s34
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_headline.py tests/test_gpu_rollout.py tests/test_gpu_parity.py tests/test_gpu_fused_step.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name lib handoff bpc
  if [ $2 = base ]; then L=""; else L="$PWD/_variants/librtenv_$2.so"; fi
  RT_LIB_PATH=$L RT_DENSE_PERSIST=$4 timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --no-update --dense-handoff $3 > $O/b_$1.json 2> $O/b_$1.err || { tail -20 $O/b_$1.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$1.json')); print('$1', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', round(d['roofline']['frac'],3))"
}
run kg1_ev kg1 0 6 && run kg8_ev base 0 6 && run kg4_ev kg4 0 6 && run kg8_dev6 base 1 6 && run kg8_dev4 base 1 4 && run kg8_dev3 base 1 3 && run kg1_ev_b kg1 0 6 && run kg8_ev_b base 0 6
echo ALLDONE
