#!/bin/bash
# r04 session 24: rocprofv3 kernel summary of the configs[3] vision bench (f32)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s24
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --vision --no-cpu --no-c3d > $O/vision_prof.json 2> $O/vision_prof.err || { tail -20 $O/vision_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/vision_kernel_stats.csv
rm -rf $O/prof
echo ALLDONE
