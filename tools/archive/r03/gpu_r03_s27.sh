#!/bin/bash
# r03 session 27: conv1 forward in bf16x3 (packed ring, 16x16x32 bf16 MFMA): C3D tests, stage timing, vision A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s27
mkdir -p $O
timeout -k 10 200 python -u tools/c3d_prec_err.py $O/prec_err.json > $O/prec_err.log 2>&1 || { tail -30 $O/prec_err.log; exit 1; }
cat $O/prec_err.log
timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-update --steps 8 --warmup 4 > $O/bench_c3d.json 2> $O/bench_c3d.err || { tail -20 $O/bench_c3d.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_c3d.json'))['c3d_mfma']
print('conv1 f32 fwd', round(d['stages']['conv1']['forward_ms'],3), 'train', round(d['stages']['conv1']['train_forward_ms'],3))
print('bf16x3', {k: (round(v,4) if isinstance(v,float) else v) for k,v in d['bf16x3'].items() if k!='note'})
print('train pass f32', round(d['train_pass']['ms'],3))"
for p in f32 bf16x3; do
  timeout -k 10 300 python -u bench.py --vision --no-cpu --no-c3d --conv-precision $p > $O/vision_$p.json 2> $O/vision_$p.err || { tail -20 $O/vision_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision_$p.json'))
print('vision $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s')"
done
echo ALLDONE
