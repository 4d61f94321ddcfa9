#!/bin/bash
# r05 session 25: conv1's sparse weight gradient reading each patch row as
# one aligned ds_read_b64 (from the plane ring or its x-shifted copy) + one
# ds_read_b32 (in-tree) vs three b32 reads (head): C3D gates, stage times x2,
# vision f32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s25
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py tests/test_gpu_configs.py tests/test_gpu_vision.py > $O/pytest_c3d.log 2>&1 || { tail -40 $O/pytest_c3d.log; exit 1; }
tail -1 $O/pytest_c3d.log
for i in 1 2; do
for v in base head; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 tools/c3d_stage_times.py > $O/stages_${v}_$i.txt 2> $O/stages_${v}_$i.err || { tail -20 $O/stages_${v}_$i.err; exit 1; }
  echo "== $v $i"; grep -v "^{" $O/stages_${v}_$i.txt | grep "f32" | grep -v bf16 | head -1
done
done
timeout -k 10 400 python3 bench.py --vision --no-cpu --no-c3d --conv-precision f32 > $O/vision_f32.json 2> $O/vision_f32.err || { tail -20 $O/vision_f32.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/vision_f32.json'))
print('vision f32: rollout', round(d['value']), 'minibatch ms', round(d['ppo_update_ms'],2), 'iteration', round(d['train_env_steps_per_s']))"
echo ALLDONE
