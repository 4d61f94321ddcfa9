#!/bin/bash
# r05 session 20: ppo_update.hip (ppons) and rtenv.hip (rtns) built without
# the SLP vectorizer vs the in-tree build: update and rollout tests on each,
# bench (no CPU / C3D) alternated x2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s20
mkdir -p $O
RT_LIB_PATH=_variants/librtenv_ppons.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trainer.py > $O/pytest_ppons.log 2>&1 || { tail -40 $O/pytest_ppons.log; exit 1; }
tail -1 $O/pytest_ppons.log
RT_LIB_PATH=_variants/librtenv_rtns.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_headline.py tests/test_gpu_parity.py > $O/pytest_rtns.log 2>&1 || { tail -40 $O/pytest_rtns.log; exit 1; }
tail -1 $O/pytest_rtns.log
for i in 1 2; do
for v in base ppons rtns; do
  L=ppo-radiotherapy_amd/librtenv.so; [ $v != base ] && L=_variants/librtenv_$v.so
  RT_LIB_PATH=$L timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/b_${v}_$i.json 2> $O/b_${v}_$i.err || { tail -20 $O/b_${v}_$i.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/b_${v}_$i.json')); s=d['steady_state']
print('$v $i value', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'upd us', round(d['ppo_update_ms']*1000,2), 'bf16x3', round(d['ppo_update_ms_bf16x3']*1000,2), 'incr', round(d['other_step_mode']['env_steps_per_s']/1e6,2), 'train', round(d['train_env_steps_per_s']/1e6,3))"
done
done
echo ALLDONE
