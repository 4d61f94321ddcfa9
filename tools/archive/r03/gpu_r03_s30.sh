#!/bin/bash
# r03 session 30: full GPU suite + smoke; C3D stage timing in f32 and bf16x3; vision A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s30
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-update --steps 8 --warmup 4 > $O/bench_c3d.json 2> $O/bench_c3d.err || { tail -20 $O/bench_c3d.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_c3d.json'))['c3d_mfma']
r=lambda x: round(x,3)
print('f32 fwd', r(d['forward']['ms']), 'train', r(d['train_pass']['ms']))
b=d['bf16x3']; print('bf16x3 fwd', r(b['forward_ms']), 'train', r(b['train_pass_ms']), 'dmax', b['max_abs_diff_vs_f32'])
print({k: {kk: r(vv) for kk,vv in v.items() if kk.endswith('_ms')} for k,v in b['stages'].items()})"
for p in bf16x3 f32; do
  timeout -k 10 300 python -u bench.py --vision --no-cpu --no-c3d --conv-precision $p > $O/vision_$p.json 2> $O/vision_$p.err || { tail -20 $O/vision_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision_$p.json'))
print('vision $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s')"
done
echo ALLDONE
