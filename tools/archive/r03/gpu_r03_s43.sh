#!/bin/bash
# r03 session 43 (final tree: suite, smoke, rehearsal, bench, kernel stats): full GPU suite, smoke, 2-rank rehearsal of the N>1 bench path,
# the default bench, and a kernel-trace summary of the same bench command
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s43
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --rehearse-same-device --no-cpu --no-c3d --steps 16 --warmup 4 > $O/rehearse2.json 2>$O/rehearse2.err || { tail -30 $O/rehearse2.err; exit 1; }
python -c "import json; d=json.load(open('$O/rehearse2.json')); print('rehearse2', d['n_gpus'], round(d['value']/1e6,3), 'M', d['config']['parallelism'])"
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms frac', round(r['frac'],3), 'kernel_ms', round(r['kernel_ms'],4), 'upd', round(d['ppo_update_ms']*1000,1), 'us')"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --no-cpu --no-steady --no-c3d > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
find $O/prof -name "*.db" -delete
head -6 $O/kernel_stats.csv | cut -c1-160
echo ALLDONE
