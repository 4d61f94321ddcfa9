#!/bin/bash
# r04 session 4: configs[3] vision bench (f32 and bf16x3 products) with the
# Winograd forward / data gradient, plus a rocprofv3 kernel summary of one
# f32 vision bench (where a minibatch step goes now)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s4
mkdir -p $O
for p in f32 bf16x3; do
  timeout -k 10 300 python -u bench.py --vision --no-cpu --conv-precision $p > $O/vision_$p.json 2> $O/vision_$p.err || { tail -20 $O/vision_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision_$p.json'))
print('vision $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s; c3d train pass f32', round(d['c3d_mfma']['train_pass']['ms'],3), 'bf16x3', round(d['c3d_mfma']['bf16x3']['train_pass_ms'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --vision --no-cpu --no-c3d > $O/vision_prof.json 2> $O/vision_prof.err || { tail -20 $O/vision_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/vision_kernel_stats.csv
rm -rf $O/prof
head -14 $O/vision_kernel_stats.csv | cut -d, -f1-5 | cut -c1-150
echo ALLDONE
