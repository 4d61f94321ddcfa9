#!/bin/bash
# r05 session 9: Winograd transforms on the packed f32 pipe (in-tree: input
# and output transforms; pkout: output side only; head: the committed
# kernels): C3D gates on the in-tree build, stage times of all three, vision f32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s9
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_configs.py > $O/pytest_c3d.log 2>&1 || { tail -40 $O/pytest_c3d.log; exit 1; }
tail -1 $O/pytest_c3d.log
for v in base pkout head; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_$v.txt 2> $O/stages_$v.err || { tail -20 $O/stages_$v.err; exit 1; }
  echo "== $v"; grep -v "^{" $O/stages_$v.txt | grep "f32" | head -4
done
for v in base head; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_$v.json 2> $O/vision_$v.err || { tail -20 $O/vision_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/vision_$v.json'))
print('$v vision f32: rollout', round(d['value']), 'minibatch ms', round(d['ppo_update_ms'],2), 'iteration', round(d['train_env_steps_per_s']))"
done
echo ALLDONE
