# pipelined dense rollout: env groups 2/3/4 (rollout parity, then two bench passes each)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-groups}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_rollout.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_rollout.log 2>&1 || { tail -20 $OUT/pytest_rollout.log; exit 1; }
tail -2 $OUT/pytest_rollout.log
for pass in 1 2; do
  for g in 2 3 4; do
    timeout -k 10 200 python -u bench.py --no-cpu --no-update --no-c3d --rollout-groups $g ${EXTRA} > $OUT/b_g${g}_p${pass}.json 2> $OUT/b_g${g}_p${pass}.err || exit 1
    python -c "import json,sys; d=json.loads(open('$OUT/b_g${g}_p${pass}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('g=$g pass=$pass', round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms kdense/launch',round(r['kernel_ms'],4),'step_frac',round(r['step_frac_of_hbm'],3), 'steady', round(d.get('steady_state',{}).get('env_steps_per_s',0)/1e6,3))"
  done
done
