#!/bin/bash
# r03 session 44: configs[3] vision bench on the final tree (f32 and bf16x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s44
mkdir -p $O
for p in bf16x3 f32; do
  timeout -k 10 300 python -u bench.py --vision --no-cpu --conv-precision $p > $O/vision_$p.json 2> $O/vision_$p.err || { tail -20 $O/vision_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision_$p.json'))
print('vision $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s; c3d train pass f32', round(d['c3d_mfma']['train_pass']['ms'],3), 'bf16x3', round(d['c3d_mfma']['bf16x3']['train_pass_ms'],3))"
done
echo ALLDONE
