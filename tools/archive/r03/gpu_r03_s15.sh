#!/bin/bash
# r03 session 15: bf16x3 layer products in k_ppo_grad_mfma -- update tests at unchanged tolerances, then update A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s15
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trainer.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest.log | grep -E "bf16x3|fused-" ; tail -1 $O/pytest.log
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --steps 16 --warmup 4 > $O/u.json 2>$O/u.err || { tail $O/u.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/u.json').read().strip().splitlines()[-1]); print('f32', round(d['ppo_update_ms']*1000,2), 'bf16x3', round(d['ppo_update_ms_bf16x3']*1000,2), 'us/minibatch', round(d['train_env_steps_per_s']/1e6,3), 'M train')"
done
