# PPO grad kernel A/B: merged one-wave-per-SIMD (default) vs actor/critic pairs (RT_PPO_GRAD_KERNEL=pair)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-ukab}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_dp.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for pass in 1 2; do
  for k in merged pair; do
    if [ $k = pair ]; then export RT_PPO_GRAD_KERNEL=pair; else unset RT_PPO_GRAD_KERNEL; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady > $OUT/b_${k}_p${pass}.json 2> $OUT/b_${k}_p${pass}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/b_${k}_p${pass}.json').read().strip().splitlines()[-1]); u=d['update_mfma']; print('$k pass $pass update_us', round(d['ppo_update_ms']*1e3,2), 'updates/s', round(d['ppo_updates_per_s']), 'train', round(d['train_env_steps_per_s']/1e6,3), 'M mfma frac', round(u['frac'],3))"
  done
done
