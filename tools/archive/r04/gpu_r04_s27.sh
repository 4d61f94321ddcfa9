#!/bin/bash
# r04 session 27: the dose-turn hand-off published by k_dense_persist itself (the
# last block stores the turn number) and a hipStreamWaitValue64 before the next
# turn instead of an event (variant td1): parity, A/B vs the product build,
# three runs each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s27
mkdir -p $O
RT_LIB_PATH=_variants/librtenv_td1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for rep in 1 2 3; do
for v in prod td1; do
  if [ $v = prod ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=_variants/librtenv_$v.so; fi
  timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; s=d['steady_state']; print('$v', $rep, 'value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],4), 'timed', round(r['timed_pass_ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'kms', {k: round(x,4) for k,x in r['kernel_ms_all'].items()})"
done
done
echo ALLDONE
