#!/bin/bash
# r03 session 32: configs[4]'s per-GPU share (vision C3D, 128^3, 512 envs) in f32 and bf16x3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s32
mkdir -p $O
for p in bf16x3 f32; do
  timeout -k 10 400 python -u bench.py --vision --grid 128 --no-cpu --no-c3d --conv-precision $p > $O/vision128_$p.json 2> $O/vision128_$p.err || { tail -20 $O/vision128_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision128_$p.json'))
print('vision128 $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],1), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s')"
done
echo ALLDONE
