# PPO update: trainer/DP parity tests, then update timing (two bench passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-upd}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for pass in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady > $OUT/b_p${pass}.json 2> $OUT/b_p${pass}.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/b_p${pass}.json').read().strip().splitlines()[-1]); u=d['update_mfma']; print('pass $pass rollout', round(d['value']/1e6,3),'M  update_ms', round(d['ppo_update_ms']*1e3,2),'us  updates/s', round(d['ppo_updates_per_s']), ' train', round(d['train_env_steps_per_s']/1e6,3), 'M  mfma frac', round(u['frac'],3))"
done
