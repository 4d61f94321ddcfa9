#!/bin/bash
# r04 session 35: does the bench's per-step time depend on the window length
# (a per-call cost) or on what precedes the window (the update)?  bench at
# K = 20, 64, 128, and K = 20 without the warmup update
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s35
mkdir -p $O
for k in 20 64 128; do
  timeout -k 10 200 python3 bench.py --gpus 1 --steps $k --warmup 5 --no-cpu --no-c3d > $O/bench_$k.json 2> $O/bench_$k.err || { tail -30 $O/bench_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$k.json')); s=d['steady_state']; print('K', $k, 'value ms', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), [round(4096*1000/x,4) for x in s['windows_env_steps_per_s']])"
done
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/bench_noupd.json 2> $O/bench_noupd.err || { tail -30 $O/bench_noupd.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_noupd.json')); s=d['steady_state']; print('K 20 no update: value ms', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4))"
echo ALLDONE
