#!/bin/bash
# r04 session 23: compact-vision render reading the stored doses straight from
# the trainer's store (rt_env_set_render_source): vision parity + trainer,
# configs[3] vision bench f32 and bf16x3
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s23
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_vision.py tests/test_gpu_trainer.py tests/test_gpu_binding.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for p in f32 bf16x3; do
  timeout -k 10 300 python -u bench.py --vision --no-cpu --conv-precision $p > $O/vision_$p.json 2> $O/vision_$p.err || { tail -20 $O/vision_$p.err; exit 1; }
  python -c "
import json; d=json.load(open('$O/vision_$p.json'))
print('vision $p: rollout', round(d['value']), 'env steps/s; minibatch', round(d['ppo_update_ms'],2), 'ms; iteration', round(d['train_env_steps_per_s']), 'env steps/s')"
done
echo ALLDONE
