#!/bin/bash
# r04 session 1: the driver's exact bench command twice (variance), then one
# rocprofv3 kernel trace of the same command (program after --), kept as CSV
# so the value pass and the instrumented pass can be cut apart.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s1
mkdir -p $O
for i in 1 2; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_$i.json')); r=d['roofline']; print('bench', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'timed', round(r['timed_pass_ms_per_step'],4), 'steady', round(d['steady_state']['ms_per_step'],4))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv
find $O/prof -name "*.db" -delete
rm -rf $O/prof
ls -la $O
echo ALLDONE
