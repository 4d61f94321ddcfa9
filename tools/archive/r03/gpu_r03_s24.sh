#!/bin/bash
# r03 session 24: kernel traces of the dense rollout, events vs device hand-off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s24
mkdir -p $O
for h in 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_h$h -o run --output-format csv -- python3 bench.py --no-cpu --no-c3d --no-steady --no-update --steps 16 --warmup 4 --dense-handoff $h > $O/b_h$h.json 2> $O/b_h$h.err || { tail -20 $O/b_h$h.err; exit 1; }
  f=$(find $O/prof_h$h -name "*kernel_trace.csv" | head -1); cp "$f" $O/trace_h$h.csv
  python3 tools/handoff_timeline.py $O/trace_h$h.csv 700 > $O/timeline_h$h.txt
  head -20 $O/timeline_h$h.txt
done
find $O -name "*.db" -delete
echo ALLDONE
