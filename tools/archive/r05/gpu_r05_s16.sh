#!/bin/bash
# r05 session 16: BASELINE configs[4]'s per-GPU share on one GPU (vision C3D,
# 128^3, 512 envs, num_steps 8), f32
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s16
mkdir -p $O
timeout -k 10 900 python3 bench.py --vision --grid 128 --num-steps 8 --no-cpu --no-c3d --conv-precision f32 > $O/vision128_f32.json 2> $O/vision128_f32.err || { tail -20 $O/vision128_f32.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/vision128_f32.json'))
print('vision 128^3 f32: rollout', round(d['value']), 'env steps/s', round(d['ms_per_step'],2), 'ms/step; minibatch ms', round(d['ppo_update_ms'],1), 'iteration', round(d['train_env_steps_per_s']), d['config'])"
echo ALLDONE
