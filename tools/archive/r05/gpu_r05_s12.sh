#!/bin/bash
# r05 session 12: each dose turn as two launches, the next group's turn
# released by an event after the first (its hand-off under the second):
# variants sNN = NN % of the group's envs in the first launch (b2: second
# launch at 2 blocks per CU); rollout tests on s90, then value / steady x2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s12
mkdir -p $O
RT_LIB_PATH=_variants/librtenv_s90.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_headline.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in base s70 s80 s90 s95 s90b2; do
    L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
    RT_LIB_PATH=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/b_${v}_$i.json')); s=d['steady_state']
print('$v $i value', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), round(s['env_steps_per_s']/1e6,3))"
  done
done
echo ALLDONE
