#!/bin/bash
# round 6: where the per-call cost of the driver's value window goes on the
# final tree (kernel + HIP runtime trace of the driver's bench command; no PMC)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_calltrace; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --hip-runtime-trace -d $O/tr -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_tr.json 2> $O/bench_tr.err || { tail -20 $O/bench_tr.err; exit 1; }
python3 tools/call_cost_trace.py $O/tr 20 > $O/call_cost.txt 2>&1; cat $O/call_cost.txt | head -60
rm -rf $O/tr
echo ALLDONE
