#!/bin/bash
# r03 session 3: full GPU suite + smoke; the update A/B (fused reduce+Adam vs
# the 3-kernel step), the default bench line and its kernel stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for v in 0 1 0 1; do
  RT_PPO_FUSED_ADAM=$v timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady > $O/ab_$v.json 2>$O/ab.err || { tail $O/ab.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/ab_$v.json').read().strip().splitlines()[-1]); print('FUSED_ADAM=$v', d['ppo_update_ms']*1000, 'us/minibatch', d['value'], d['train_env_steps_per_s'])"
done
timeout -k 10 300 python -u bench.py > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
tail -c 1500 $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bkt -o run --output-format csv -- python3 bench.py --no-cpu > $O/bench_kt.json 2>$O/bench_kt.err || { tail $O/bench_kt.err; exit 1; }
find $O -name "*.db" -delete
echo ALLDONE
