#!/bin/bash
# r04 session 8: the dense rollout's k_dense turns on a dedicated dose stream
# (back to back in launch order) instead of a ring of event hand-offs between
# the group streams; optional CU partition (chain streams on 1 CU in 8 / 4 of
# each XCD, the dose stream on the rest).  Rollout parity, then the sweep vs
# the event-ring builds (b6u8 / b5u8), two runs each, staggered phases
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2; do
for v in b6u8 b5u8 q0b6 q0b5 q8b6 q4b6 q8b5 q4b8; do
  RT_LIB_PATH=tools/_variants/$v.so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; s=d['steady_state']; print('$v', $rep, 'value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'kms', {k: round(x,4) for k,x in r['kernel_ms_all'].items()}, 'iso', round(r['isolated']['kernel_ms'],4))"
done
done
echo ALLDONE
