# pipelined dense rollout: k_dense turns (default) vs free-running groups (RT_PIPE_SERIAL=0); two passes each
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-serial}
mkdir -p $OUT
for pass in 1 2; do
  for v in 1 0; do
    RT_PIPE_SERIAL=$v timeout -k 10 200 python -u bench.py --no-cpu --no-update --no-c3d > $OUT/b_s${v}_p${pass}.json 2> $OUT/b_s${v}_p${pass}.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/b_s${v}_p${pass}.json').read().strip().splitlines()[-1]); r=d['roofline']; print('serial=$v pass $pass', round(d['value']/1e6,3),'M', round(d['ms_per_step'],4),'ms kdense', round(r['kernel_ms'],4), 'steady', round(d['steady_state']['env_steps_per_s']/1e6,3))"
  done
done
