# PPO grad kernel: static wave priority variants (RT_LIB_PATH builds from tools/build_variant.py), two passes
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-prio}
mkdir -p $OUT
for pass in 1 2; do
  for v in base prio1 prio2; do
    if [ $v = base ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$GRAFT_REPO_ROOT/_variants/librtenv_$v.so; fi
    timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady > $OUT/b_${v}_p${pass}.json 2> $OUT/b_${v}_p${pass}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/b_${v}_p${pass}.json').read().strip().splitlines()[-1]); print('$v pass $pass update_us', round(d['ppo_update_ms']*1e3,2), 'train', round(d['train_env_steps_per_s']/1e6,3))"
  done
done
