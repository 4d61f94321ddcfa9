#!/bin/bash
# r03 session 25: device hand-off without fences (nt loads / sc1 stores): rollout tests, A/B, trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s25
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_rollout.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in "0 2" "1 2" "1 3" "1 4" "0 2" "1 2"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --no-cpu --no-c3d --no-steady --no-update --dense-handoff $1 --rollout-groups $2 > $O/b_h$1_g$2.json 2> $O/b_h$1_g$2.err || { tail -20 $O/b_h$1_g$2.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_h$1_g$2.json')); r=d['roofline']; print('handoff $1 groups $2', round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), 'ms', r['kernel'], round(r['frac'],3), round(r['step_frac_of_hbm'],3))"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_h1 -o run --output-format csv -- python3 bench.py --no-cpu --no-c3d --no-steady --no-update --steps 16 --warmup 4 --dense-handoff 1 > $O/bt_h1.json 2> $O/bt_h1.err || { tail -20 $O/bt_h1.err; exit 1; }
f=$(find $O/prof_h1 -name "*kernel_trace.csv" | head -1); cp "$f" $O/trace_h1.csv
python3 tools/handoff_timeline.py $O/trace_h1.csv 1000 > $O/timeline_h1.txt
grep -v "k_probe\|at::native\|rocclr_copy\|rocclr_fill" $O/timeline_h1.txt | head -50
find $O -name "*.db" -delete
echo ALLDONE
