#!/bin/bash
# r05 session 10: dense rollout with group 0 on the caller's stream (in-tree)
# vs the fork of every group onto library streams (fork2 = HEAD rtenv.hip):
# rollout tests, the driver's bench command alternated x3, one call-cost trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s10
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_headline.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in base fork2; do
    L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
    RT_LIB_PATH=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_${v}_$i.json')); s=d['steady_state']
print('$v $i value', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'vs_value', round(s['vs_value'],4))"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/tr -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_tr.json 2> $O/bench_tr.err || { tail -20 $O/bench_tr.err; exit 1; }
python3 tools/call_cost_trace.py $O/tr 20 > $O/call_cost.txt; head -45 $O/call_cost.txt
rm -rf $O/tr
echo ALLDONE
