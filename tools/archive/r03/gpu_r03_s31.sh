#!/bin/bash
# r03 session 31: bf16x3 also in the grouped data gradient: C3D tests, timing, vision A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s31
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_c3d.py > $O/pytest_c3d.log 2>&1 || { tail -60 $O/pytest_c3d.log; exit 1; }
tail -2 $O/pytest_c3d.log
timeout -k 10 200 python -u tools/c3d_prec_err.py $O/prec_err.json > $O/prec_err.log 2>&1 || { tail -30 $O/prec_err.log; exit 1; }
grep -v Warning $O/prec_err.log | grep "^(" 
timeout -k 10 300 python -u bench.py --no-cpu --no-steady --no-update --steps 8 --warmup 4 > $O/bench_c3d.json 2> $O/bench_c3d.err || { tail -20 $O/bench_c3d.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_c3d.json'))['c3d_mfma']
print('stages f32', {k: {kk: round(vv,3) for kk,vv in v.items() if kk.endswith('_ms')} for k,v in d['stages'].items()})
b=d['bf16x3']; print('bf16x3 fwd', round(b['forward_ms'],3), 'train', round(b['train_pass_ms'],3), 'dmax', b['max_abs_diff_vs_f32']); print({k: {kk: round(vv,3) for kk,vv in v.items() if kk.endswith('_ms')} for k,v in b['stages'].items()})
print('train pass f32', round(d['train_pass']['ms'],3))"
for p in f32 bf16x3; do
  timeout -k 10 300 python -u bench.py --vision --no-cpu --no-c3d --conv-precision $p > $O/vision_$p.json 2> $O/vision_$p.err || { tail -20 $O/vision_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision_$p.json'))
print('vision $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s')"
done
echo ALLDONE
