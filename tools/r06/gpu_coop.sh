#!/bin/bash
# round 6: k_ppo_reduce_adam as a cooperative launch (co-residency guaranteed
# by the runtime) against the plain launch: trainer gates, then the update line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_coop; mkdir -p $O
RT_PPO_COOP=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trainer.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in 0 1 0 1; do
  RT_PPO_COOP=$m timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-steady > $O/b$m.json 2> $O/b$m.err || { tail -20 $O/b$m.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads([l for l in open('$O/b$m.json') if l.startswith('{')][-1])
print('coop $m', 'update us %.2f' % (d['ppo_update_ms']*1e3), 'bf16x3 %.2f' % (d['ppo_update_ms_bf16x3']*1e3), 'coll %.2f' % (d['ppo_update_ms_collective_path']*1e3), 'value %.3f M' % (d['value']/1e6))
"
done
echo ALLDONE
